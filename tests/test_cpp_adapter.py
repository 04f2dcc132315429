"""The C++ drop-in adapter (include/pvac_hip.hpp): built by __graft_entry__.build() into
tests/cpp/build/test_adapter; on the GPU box it replays the reference's golden streams through the
by-value API (ct_add/ct_sub/ct_scale/ct_mul with sigma/chains/fp, enc_value/dec_value, .ct load/save) and compares byte for byte."""
import json
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "tests", "cpp", "build", "test_adapter")
GOLD = os.path.join(ROOT, "tests", "golden")


def test_adapter_binary_links():
    """CPU-side: the adapter test program was built and resolves libpvac_hip.so in-tree."""
    if not os.path.exists(EXE):
        pytest.skip("tests/cpp not built (run __graft_entry__.build())")
    out = subprocess.run(["ldd", EXE], capture_output=True, text=True).stdout
    line = [l for l in out.splitlines() if "libpvac_hip.so" in l]
    assert line and "not found" not in line[0]
    assert os.path.join("pvac_hfhe_cppbyv_amd", "lib") in os.path.normpath(line[0].split("=>")[1])


@pytest.mark.gpu
def test_adapter_against_golden():
    assert os.path.exists(EXE), "tests/cpp/build/test_adapter missing: build() must compile it"
    with open(os.path.join(GOLD, "ref", "manifest.json")) as f:
        man = json.load(f)
    with open(os.path.join(GOLD, "ref", "enc_manifest.json")) as f:
        vs = ",".join(str(e["v"]) for e in json.load(f)["enc"])
    with open(os.path.join(GOLD, "ref", "encd_manifest.json")) as f:
        ds = ",".join(f"{int(c['kind'] == 'zero')}:{c['v']}:{c['depth']}" for c in json.load(f)["cases"])
    r = subprocess.run([EXE, GOLD, str(man["canon_tag"]), man["H_digest"], vs, ds], capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "checks passed" in r.stdout
