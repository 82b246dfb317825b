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
    mock cloud with g++ alone, with the solver calls spelled exactly as laser_odometry.cpp:183-229
    spells them (solver.h:84-139 argument lists: no extra context argument)."""
    src = tmp_path / "adapter.cpp"
    src.write_text(f'''
#include <array>
#include <memory>
#include <vector>
#include "{ROOT / "include" / "imls_icp_hip.hpp"}"
struct Pt {{ float x, y, z, _p0, normal_x, normal_y, normal_z, _p1, intensity, curvature, _p2, _p3; }};
struct Cloud {{ std::vector<Pt> points; size_t size() const {{ return points.size(); }}
  void push_back(const Pt& p) {{ points.push_back(p); }} void clear() {{ points.clear(); }} }};
struct Mat4 {{ double m[16]; double& operator()(int r, int c) {{ return m[r * 4 + c]; }} }};
using namespace imls_hip;
int main() {{
  IMLSICPMatcherHip m;                       // was: IMLSICPMatcher matcher;
  auto a = std::make_shared<Cloud>(); auto b = std::make_shared<Cloud>();
  m.setSourcePointCloud(a); m.setTargetPointCloud(a);
  m.setParameters(30, 1.0, 3.0, 1.0, 0.8, false, true, false, 50, 0.2, 0.6, 10, 20, true, 30.0, "out/");
  m.ProjSourcePtToSurface(a, b, std::string("0"), 0);
  std::vector<std::array<double,3>> s, d, n; Mat4 D; std::vector<double> w; std::string ts = "0";
  bool ok = SolveMotionEstimationProblemLS(s, d, n, D, ts, 0.02);
  ok = ok && SolveMotionEstimationProblemWeightedLS(s, d, n, D, w, ts);
  ok = ok && SolveMotionEstimationProblemRANSAC(s, d, n, D, ts, 5000, 0.8, 0.95, 0.648, "DRPM", 0.02, 0.05, 0.02, 0.05);
  ok = ok && SolveMotionEstimationProblemDRPM(s, d, n, D, w, ts, 0.05, 0.02, 0.05);
  m.planeICPProj(a, b, 1.5, false, 0.8, true, 30.0);
  double P[16]; m.registerFrame(P);
  (void)ok; return 0; }}
''')
    subprocess.run(["g++", "-std=c++17", "-Wall", "-Werror", "-fsyntax-only", f"-I{ROOT / 'include'}", str(src)],
                   check=True)


def test_type_swap_program_links_against_the_library():
    """tests/cpp/type_swap (the reference loop over the adapter) is built by build() and links
    libimls_gpu.so; without a GPU it must fail loudly (no CPU fallback), not compute."""
    exe = ROOT / "tests" / "cpp" / "type_swap"
    if not exe.exists():
        subprocess.run(["make", "-C", str(exe.parent)], check=True)
    out = subprocess.run(["ldd", str(exe)], capture_output=True, text=True, check=True).stdout
    assert "libimls_gpu.so" in out and "not found" not in out
    import torch
    if not torch.cuda.is_available():
        r = subprocess.run([str(exe), "LS", "3", "/nonexistent", "/nonexistent"], capture_output=True, text=True)
        assert r.returncode != 0


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


def test_library_reads_no_tuning_environment():
    """Runtime tuning goes through imls_set_option only (ADVICE/VERDICT r04): the only IMLS_*
    environment name left in the product library is the host-side trace switch IMLS_DEBUG_HOST."""
    data = _abi.LIB_PATH.read_bytes()
    import re
    names = set(re.findall(rb"IMLS_[A-Z0-9_]+", data))
    assert names <= {b"IMLS_DEBUG_HOST"}, names


def test_option_ids_match_header():
    """imls_option / imls_traversal enum values in include/imls_gpu.h equal the Python mirror."""
    text = HEADER.read_text()
    import re
    for name, val in _abi.OPTION_IDS.items():
        m = re.search(rf"IMLS_OPT_{name.upper()}\s*=\s*(\d+)", text)
        assert m and int(m.group(1)) == val, name
    for name in ("AUTO", "PACKETS", "WAVE_PER_QUERY", "LANE"):
        m = re.search(rf"IMLS_TRAVERSAL_{name}\s*=\s*(\d+)", text)
        assert m and int(m.group(1)) == getattr(_abi, f"IMLS_TRAVERSAL_{name}"), name
