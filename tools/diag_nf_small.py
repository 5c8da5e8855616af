"""Diagnostics (development): the device build's small-task sizes on cfg5 frames."""
import sys
import numpy as np
sys.path.insert(0, ".")
sys.path.insert(0, "tests")
import dynamic_direct_lidar_odometry_amd as P
from dynamic_direct_lidar_odometry_amd import TARGET, scene
from test_gpu_nftree import _TASK, _ctl

frames = scene.loop_sequence(64, 2048, 0, 3, device=0)[0]
for f in frames:
    c = P.Context(0)
    c.set_target(f)
    vind, info, st, raw = c.nfbuild_debug(TARGET, stop=-1, scratch_bytes=1 << 23)
    ctl = _ctl(raw)
    Lmax, max_task, max_pend, max_small = (int(x) for x in info[:4])
    small = raw[info[7]:info[7] + _TASK.itemsize * max_small].view(_TASK)[:ctl["nsmall"]]
    cnt = np.sort(small["count"])
    print("n", len(f), "Lmax", Lmax, "status", st.tolist(), "ntask", ctl["ntask"][:Lmax + 1], "nsmall", ctl["nsmall"],
          "largest", cnt[-8:].tolist(), "over4096", int((cnt > 4096).sum()), "sum", int(cnt.sum()))
    c.close()
