"""CPU tests of the C-ABI boundary: the library loads, exports every symbol include/imls_gpu.h
declares, the ctypes mirror matches the C struct layout, and the product path fails loudly (no
CPU fallback) when no GPU is present."""
import ctypes as C
import pathlib
import re
import subprocess

import pytest

from planetary_lidar_odometry_amd import _abi, config

ROOT = pathlib.Path(__file__).resolve().parent.parent
HEADER = ROOT / "include" / "imls_gpu.h"


def declared_functions():
    text = re.sub(r"/\*.*?\*/", "", HEADER.read_text(), flags=re.S)
    return sorted(set(re.findall(r"^\s*[\w\s\*]+?\b(imls_\w+)\s*\(", text, flags=re.M)))


def test_library_exports_every_declared_symbol():
    lib = _abi.load_library()
    names = declared_functions()
    assert len(names) >= 20
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert set(names) == set(_abi.ABI_SYMBOLS)
    out = subprocess.run(["nm", "-D", "--defined-only", str(_abi.LIB_PATH)], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r"\bT (imls_\w+)", out))
    assert set(names) <= exported


def test_abi_version_and_defaults():
    lib = _abi.load_library()
    assert lib.imls_abi_version() == 1
    p = _abi.ImlsParams()
    lib.imls_default_params(C.byref(p))
    assert p.as_dict() == _abi.default_params().as_dict()
    assert p.as_dict() == config.params_from_config(config.load()).as_dict()


def test_struct_layout_matches_c(tmp_path):
    fields = [f for f, _ in _abi.ImlsParams._fields_]
    prog = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void){",
            'printf("%zu\\n", sizeof(imls_params));', 'printf("%zu\\n", sizeof(imls_iter_trace));']
    prog += [f'printf("%zu\\n", offsetof(imls_params, {f}));' for f in fields]
    prog += ["return 0;}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(prog))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == C.sizeof(_abi.ImlsParams)
    assert vals[1] == C.sizeof(_abi.ImlsIterTrace)
    for f, off in zip(fields, vals[2:]):
        assert getattr(_abi.ImlsParams, f).offset == off, f


@pytest.mark.parametrize("ctype,cname", [(_abi.ImlsPcaParams, "imls_pca_params"),
                                          (_abi.ImlsSampleParams, "imls_sample_params")])
def test_producer_struct_layouts_and_defaults(tmp_path, ctype, cname):
    fields = [f for f, _ in ctype._fields_]
    prog = ["#include <stdio.h>", "#include <stddef.h>", f'#include "{HEADER}"', "int main(void){",
            f'printf("%zu\\n", sizeof({cname}));']
    prog += [f'printf("%zu\\n", offsetof({cname}, {f}));' for f in fields]
    prog += ["return 0;}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(prog))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c11", "-o", str(exe), str(src)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert vals[0] == C.sizeof(ctype)
    for f, off in zip(fields, vals[1:]):
        assert getattr(ctype, f).offset == off, f
    lib = _abi.load_library()
    as_dict = lambda p: {f: getattr(p, f) for f in fields}
    if ctype is _abi.ImlsPcaParams:
        p = ctype()
        lib.imls_default_pca_params(C.byref(p))
        assert as_dict(p) == as_dict(_abi.default_pca_params())
    else:
        for m in (_abi.IMLS_SAMPLE_NORMAL, _abi.IMLS_SAMPLE_MAJOR_AXIS):
            p = ctype()
            lib.imls_default_sample_params(C.byref(p), m)
            assert as_dict(p) == as_dict(_abi.default_sample_params(m))


def test_cpp_adapter_header_compiles(tmp_path):
    """include/imls_icp_hip.hpp (the reference-shaped C++ adapter) compiles against a PCL-shaped
    mock cloud with g++ alone."""
    src = tmp_path / "adapter.cpp"
    src.write_text(f'''
#include <memory>
#include <vector>
#include "{ROOT / "include" / "imls_icp_hip.hpp"}"
struct Pt {{ float x, y, z, _p0, normal_x, normal_y, normal_z, _p1, intensity, curvature, _p2, _p3; }};
struct Cloud {{ std::vector<Pt> points; size_t size() const {{ return points.size(); }}
  void push_back(const Pt& p) {{ points.push_back(p); }} void clear() {{ points.clear(); }} }};
int main() {{
  imls_params p; imls_hip::IMLSICPMatcherHip m(0, nullptr);
  auto a = std::make_shared<Cloud>(); auto b = std::make_shared<Cloud>();
  m.setSourcePointCloud(a); m.setTargetPointCloud(a);
  m.ProjSourcePtToSurface(a, b, std::string("0"), 0, nullptr);
  std::vector<std::array<double,3>> s, d, n; double D[16];
  bool ok = imls_hip::SolveMotionEstimationProblemLS(m, s, d, n, D, "0", 0.02);
  m.planeICPProj(a, b, 1.5, false, 0.8, true, 30.0);
  ok = ok && imls_hip::SolveMotionEstimationProblemRANSAC(m, s, d, n, D, "0", 5000, 0.8, 0.95, 0.648, "DRPM",
                                                        0.02, 0.05, 0.02, 0.05);
  (void)ok; (void)p; return 0; }}
''')
    subprocess.run(["g++", "-std=c++17", "-fsyntax-only", str(src)], check=True)


def test_product_path_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    lib = _abi.load_library()
    assert not lib.imls_create(0, C.byref(_abi.default_params()))
    from planetary_lidar_odometry_amd import imls_icp
    with pytest.raises(_abi.ImlsError):
        imls_icp.ImlsContext()


def test_missing_library_raises(tmp_path):
    with pytest.raises(RuntimeError, match="HIP extension missing"):
        _abi.load_library(tmp_path / "nope.so")
