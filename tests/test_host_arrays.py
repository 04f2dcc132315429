"""The C++ adapter's host side without a GPU (tests/cpp/host_arrays_check.cpp): reference-shaped
Ciphers through to_host / convert_host round trip exactly (ragged shapes, with and without
sigma, plain and page-locked host arrays), and the page-locked arrays fall back to ordinary
memory when the runtime refuses to pin, leaving nothing registered."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_adapter_host_arrays(tmp_path):
    lib = os.path.join(ROOT, "pvac_hfhe_cppbyv_amd", "lib")
    if not os.path.exists(os.path.join(lib, "libpvac_hip.so")):
        pytest.skip("libpvac_hip.so not built (run __graft_entry__.build())")
    out = str(tmp_path / "host_arrays_check")
    cmd = ["g++", "-std=c++17", "-O2", "-Wall", "-Wextra", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROOT, "include"),
           "-I", "/opt/rocm/include", os.path.join(ROOT, "tests", "cpp", "host_arrays_check.cpp"), "-o", out,
           "-pthread", "-L", lib, "-lpvac_hip", "-L", "/opt/rocm/lib", "-lamdhip64", f"-Wl,-rpath,{lib}",
           "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-4000:]
    r = subprocess.run([out], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "host_arrays_check: ok" in r.stdout
