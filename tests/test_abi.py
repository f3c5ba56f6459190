"""The C-ABI library builds/loads and exports every symbol include/slat.h declares. CPU only
(no compute calls: there is no GPU here)."""
import os
import re
import subprocess


import slat
from slat import _lib as L

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    txt = open(os.path.join(ROOT, "include", "slat.h")).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(slat_[a-z0-9_]+)\s*\(", txt)))


def test_header_matches_binding_list():
    assert header_symbols() == sorted(L.EXPORTS)


def test_library_exports_every_symbol():
    out = subprocess.run(["nm", "-D", "--defined-only", L.LIB_PATH], capture_output=True, text=True, check=True).stdout
    defined = set(re.findall(r"\bT (slat_\w+)", out))
    missing = [s for s in header_symbols() if s not in defined]
    assert not missing, missing


def test_library_loads_and_reports_no_device_here():
    lib = slat.lib()
    for s in L.EXPORTS:
        assert hasattr(lib, s)
    assert lib.slat_status_string(0) == b"ok"


def test_kernels_built_for_gfx950():
    """The offload bundle inside libslat.so holds gfx950 code objects and no other GPU target."""
    blob = open(L.LIB_PATH, "rb").read()
    targets = set(re.findall(rb"hipv4-amdgcn-amd-amdhsa--(gfx[0-9a-f]+)", blob))
    assert targets == {b"gfx950"}, targets
