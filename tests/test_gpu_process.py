"""Process-level behaviour of the library's load: which HIP runtime the process binds to, and a
clean exit after the library, torch.distributed and RCCL's unique id have all been loaded.

PyTorch-ROCm bundles libamdhip64.so.7 / librccl.so.1 under the same sonames as /opt/rocm's; the first one loaded
serves the whole process.  `load()` imports torch first (when it is installed and DDLO_TORCH_FIRST is not "0"),
so a Python process that also uses torch.distributed runs both on torch's runtime; a process that sets
DDLO_TORCH_FIRST=0 and never imports torch binds to the runtime of the library's RUNPATH (/opt/rocm), as a C++
host does.  Each case runs in a fresh subprocess and must exit with status 0.
"""
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

ALIGN = r"""
import numpy as np
import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import scene
src, tgt, T = scene.s2s_pair(32, 256, 1)
c = P.Context(0, P.default_params(max_correspondence_distance=1.0))
c.set_target(tgt)
c.set_source(src)
out, res = c.align()
assert res.iterations_run > 0
"""

MAPS = r"""
hip = sorted({l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l})
print('HIP_RUNTIME', hip)
"""


def _run(code, env_extra):
    env = dict(os.environ)
    env.update(env_extra)
    env["PYTHONPATH"] = ROOT + os.pathsep + env.get("PYTHONPATH", "")
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    return p.returncode, p.stdout + p.stderr


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_library_then_torch_distributed_and_rccl_id_exit_clean():
    """The library loads (default: torch first), then torch.distributed opens a gloo group, RCCL's unique id is
    made and broadcast, a one-rank RCCL communicator aligns, and the process exits with 0."""
    code = ALIGN + r"""
import os
import torch.distributed as dist
dist.init_process_group("gloo", init_method="tcp://127.0.0.1:%d", rank=0, world_size=1)
uid = [P.comm_unique_id()]
dist.broadcast_object_list(uid, src=0)
c.set_comm(uid[0], 1, 0)
out2, res2 = c.align()
assert res2.iterations_run == res.iterations_run
c.close()
dist.destroy_process_group()
""" % _port() + MAPS
    rc, out = _run(code, {})
    print(out[-2000:])
    assert rc == 0, out[-4000:]
    assert "torch/lib" in out.split("HIP_RUNTIME", 1)[1], out[-2000:]


def test_library_without_torch_binds_rocm_runtime():
    """DDLO_TORCH_FIRST=0 and no torch anywhere: the library binds to /opt/rocm's HIP runtime (its RUNPATH),
    aligns, and the process exits with 0 without ever importing torch."""
    code = ALIGN + r"""
import sys
assert "torch" not in sys.modules
c.close()
""" + MAPS
    rc, out = _run(code, {"DDLO_TORCH_FIRST": "0"})
    print(out[-2000:])
    assert rc == 0, out[-4000:]
    rt = out.split("HIP_RUNTIME", 1)[1]
    assert "rocm" in rt and "torch" not in rt, out[-2000:]
