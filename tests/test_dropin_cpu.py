"""The C++ drop-in header (include/slat.hpp) and its test program compile here with g++ (no GPU
needed), warnings as errors; the built program links against every libslat.so symbol it uses."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INC = os.path.join(ROOT, "include")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not on PATH")
def test_header_compiles(tmp_path):
    src = tmp_path / "use.cpp"
    src.write_text('#include "slat.hpp"\n'
                   "int main() {\n"
                   "  slat::CsrMatrix a = slat::CsrMatrix::identity(4);\n"
                   "  slat::MagnusMatrix m = slat::MagnusMatrix::empty(4);\n"
                   "  slat::Csr<double> f; slat::Csr<uint64_t> g; slat::Csr<uint32_t> h;\n"
                   "  (void)a; (void)m; (void)f; (void)g; (void)h;\n"
                   "  return 0;\n}\n")
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-fsyntax-only", f"-I{INC}", str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not on PATH")
def test_dropin_program_compiles(tmp_path):
    r = subprocess.run(["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-c", f"-I{INC}",
                        os.path.join(ROOT, "tests", "cpp", "dropin.cpp"), "-o", str(tmp_path / "dropin.o")],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    nm = subprocess.run(["nm", "-u", str(tmp_path / "dropin.o")], capture_output=True, text=True).stdout
    used = {ln.split()[-1] for ln in nm.splitlines() if ln.split() and ln.split()[-1].startswith("slat_")}
    assert {"slat_spgemm_csr_u32", "slat_magnus_matmul", "slat_spgemm_csr_f64", "slat_csr_add"} <= used
    import slat  # the exported symbols the program needs are in the library
    L = slat.lib()
    for s in used:
        assert hasattr(L, s), s
