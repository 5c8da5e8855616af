"""CPU tests of the drop-in boundary: the C-ABI library loads, exports every
entry point include/ddlo_gicp.h declares, its structs have the layout the
bindings assume, and with no GPU every compute entry point fails loudly
(GICP_EHIP) instead of falling back to the CPU."""
import ctypes as C
import os
import re
import shutil
import subprocess

import numpy as np
import pytest

import dynamic_direct_lidar_odometry_amd as P

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "ddlo_gicp.h")


def declared_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?[\w\*]+\s*\**\s*(gicp_\w+)\s*\(", txt, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("gicp_ctx_create", "gicp_set_source", "gicp_set_target", "gicp_align", "gicp_compute_covariances",
                 "gicp_set_covariances", "gicp_get_covariances", "gicp_swap_source_target", "gicp_get_residuals"):
        assert must in names
    assert len(names) >= 29


def test_library_exports_every_declared_symbol():
    path = P.lib_path()
    assert os.path.exists(path), "build the library first (make lib)"
    out = subprocess.run(["nm", "-D", "--defined-only", path], check=True, capture_output=True, text=True).stdout
    exported = set(line.split()[-1] for line in out.splitlines() if line.strip())
    missing = [n for n in declared_functions() if n not in exported]
    assert not missing, f"declared but not exported: {missing}"
    L = P.load()
    for n in declared_functions():
        assert hasattr(L, n)


def test_python_binding_covers_every_symbol():
    src = open(os.path.join(ROOT, "dynamic_direct_lidar_odometry_amd", "__init__.py")).read()
    for n in declared_functions():
        assert f'"{n}"' in src, f"{n} has no ctypes signature in the binding"


STRUCT_PROBE = r"""
#include <stddef.h>
#include <stdio.h>
#include "ddlo_gicp.h"
#define F(T, m) printf(#T " " #m " %zu %zu\n", offsetof(T, m), sizeof(((T*)0)->m));
int main(void) {
  printf("gicp_params size %zu 0\n", sizeof(gicp_params));
  printf("gicp_result size %zu 0\n", sizeof(gicp_result));
  F(gicp_params, k_correspondences) F(gicp_params, max_iterations) F(gicp_params, max_correspondence_distance)
  F(gicp_params, transformation_epsilon) F(gicp_params, rotation_epsilon) F(gicp_params, lm_init_lambda_factor)
  F(gicp_params, regularization) F(gicp_params, optimizer) F(gicp_params, lm_max_iterations)
  F(gicp_params, fixed_iterations)
  F(gicp_result, converged) F(gicp_result, nr_iterations) F(gicp_result, iterations_run) F(gicp_result, lm_failed)
  F(gicp_result, lm_trials) F(gicp_result, num_correspondences) F(gicp_result, final_cost)
  F(gicp_result, final_hessian) F(gicp_result, lm_lambda) F(gicp_result, device_ms) F(gicp_result, linearize_ms)
  return 0;
}
"""


@pytest.mark.skipif(shutil.which("gcc") is None, reason="gcc not available")
def test_struct_layout_matches_ctypes(tmp_path):
    c = tmp_path / "probe.c"
    c.write_text(STRUCT_PROBE)
    exe = tmp_path / "probe"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(c), "-o", str(exe)], check=True)
    out = subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.split("\n")
    types = {"gicp_params": P.GicpParams, "gicp_result": P.GicpResult}
    for line in filter(None, out):
        t, m, off, size = line.split()
        if m == "size":
            assert C.sizeof(types[t]) == int(off), t
        else:
            fld = getattr(types[t], m)
            assert fld.offset == int(off) and fld.size == int(size), (t, m)


def test_default_params_are_the_reference_defaults():
    p = P.default_params()
    # nano_gicp_impl.hpp:58-62, lsq_registration_impl.hpp:53-60, pcl Registration defaults
    assert p.k_correspondences == 20
    assert p.max_correspondence_distance == pytest.approx(np.finfo(np.float32).max)
    assert p.transformation_epsilon == 5e-4 and p.rotation_epsilon == 2e-3
    assert p.lm_init_lambda_factor == 1e-9 and p.lm_max_iterations == 10
    assert p.regularization == P.REG_PLANE and p.optimizer == P.LEVENBERG_MARQUARDT
    assert p.max_iterations == 64 and p.fixed_iterations == 0
    assert P.load().gicp_abi_version() >= 1


def test_default_options():
    """Process-wide option defaults (gicp_set_default_option): the documented values, settable and
    restorable, out-of-range values and unknown options rejected (no device needed)."""
    assert P.get_default_option(P.OPT_TIE_ORDER) == 1
    assert P.get_default_option(P.OPT_TIE_LAZY) == 1
    assert P.get_default_option(P.OPT_TIE_PARTIAL_LEVELS) == 3
    assert P.get_default_option(P.OPT_COV_TASKS) == 0
    assert P.get_default_option(P.OPT_GRID_MAX_MB) == 0
    with P.default_option(P.OPT_GRID_MAX_MB, 150):
        assert P.get_default_option(P.OPT_GRID_MAX_MB) == 150
    with P.default_option(P.OPT_TIE_ORDER, 0):
        assert P.get_default_option(P.OPT_TIE_ORDER) == 0
    assert P.get_default_option(P.OPT_TIE_ORDER) == 1
    for opt, val in ((0, 1), (6, 1), (P.OPT_TIE_ORDER, 2), (P.OPT_TIE_PARTIAL_LEVELS, -1), (P.OPT_TIE_PARTIAL_LEVELS, 25),
                     (P.OPT_GRID_MAX_MB, -1)):
        with pytest.raises(P.GicpError):
            P.set_default_option(opt, val)


def _gpu_present():
    n = C.c_void_p()
    rc = P.load().gicp_ctx_create(0, C.byref(n))
    if rc == 0:
        P.load().gicp_ctx_destroy(n)
        return True
    return False


def test_no_gpu_fails_loudly():
    if _gpu_present():
        pytest.skip("a GPU is visible; this checks the no-GPU behaviour")
    with pytest.raises(P.GicpError) as e:
        P.Context(0)
    assert e.value.status == 5  # GICP_EHIP
    assert "device" in str(e.value).lower()


def test_null_arguments_rejected():
    L = P.load()
    assert L.gicp_ctx_create(0, None) == 1                      # GICP_EINVAL
    assert L.gicp_default_params(None) == 1
    assert L.gicp_align(None, None, None, None) == 1
    assert L.gicp_set_source(None, None, 0, 12, 1) == 1
    assert b"null" in L.gicp_last_error().lower()


def test_missing_library_raises(monkeypatch, tmp_path):
    monkeypatch.setattr(P, "_LIB", None)
    monkeypatch.setattr(P, "lib_path", lambda: str(tmp_path / "nope.so"))
    with pytest.raises(RuntimeError, match="HIP library not built"):
        P.load()


def test_product_does_not_import_the_oracle():
    pkg = os.path.join(ROOT, "dynamic_direct_lidar_odometry_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith((".py", ".hip", ".hpp", ".cpp", ".h")):
                txt = open(os.path.join(dp, f)).read()
                assert "import oracle" not in txt and "from oracle" not in txt and "liboracle" not in txt, f


def test_cpp_facade_compiles(tmp_path):
    """include/nano_gicp/nano_gicp.hpp instantiates NanoGICP<PointXYZI, PointXYZI> with every OdomNode call."""
    src = tmp_path / "f.cpp"
    src.write_text(r"""
#include "nano_gicp/nano_gicp.hpp"
using G = ddlo::NanoGICP<ddlo::PointXYZI, ddlo::PointXYZI>;
void use(G& s2s, G& s2m, ddlo::PointCloud<ddlo::PointXYZI>::ConstPtr a, ddlo::PointCloud<ddlo::PointXYZI>::ConstPtr b) {
  s2s.setCorrespondenceRandomness(10); s2s.setMaxCorrespondenceDistance(1.0); s2s.setMaximumIterations(32);
  s2s.setTransformationEpsilon(0.01); s2s.setEuclideanFitnessEpsilon(0.01); s2s.setRANSACIterations(0);
  s2s.setRANSACOutlierRejectionThreshold(1.0);
  s2s.setInputSource(a); s2s.calculateSourceCovariances(); s2s.setInputTarget(b);
  ddlo::PointCloud<ddlo::PointXYZI> out; s2s.align(out); (void)s2s.getFinalTransformation();
  s2s.swapSourceAndTarget(); s2m.registerInputSource(a); s2m.shareSourceFrom(s2s);
  s2m.setTargetCovariances(s2s.getSourceCovariances()); s2m.align(out, s2s.getFinalTransformation());
  std::vector<double> r; s2m.getResiduals(r); (void)s2m.hasConverged(); (void)s2m.getFinalHessian();
}
""")
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-Wall", "-I", os.path.join(ROOT, "include"), str(src)],
                   check=True)
