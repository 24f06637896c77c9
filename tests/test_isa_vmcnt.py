"""The packet sweep's loader (trisolve.hip k_tri_pk6) and the line sweeps'
loaders and pollers (linesweep.hip k_line2, linefill.hip k_linef) issue loads from inline asm with explicit
vmcnt waits.  Compile the device code for gfx950 and
check, on the generated assembly, that no instruction touches a VGPR that is
still the destination of an outstanding load, and that no instantiation spills
(a spill of an in-flight register would store garbage).  CPU-only: hipcc
cross-compiles, nothing runs on a GPU."""
import os
import re
import shutil
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))

HIPCC = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"


def _compile(tmp_path_factory, src):
    if not os.path.exists(HIPCC):
        pytest.skip("hipcc not available")
    out = tmp_path_factory.mktemp("isa") / (src + ".s")
    cmd = [HIPCC, "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950",
           "-I" + os.path.join(ROOT, "include"), "--cuda-device-only", "-S", "-x", "hip",
           os.path.join(ROOT, "lssp_amd", "csrc", src), "-o", str(out)]
    subprocess.run(cmd, check=True, capture_output=True)
    return str(out)


@pytest.fixture(scope="module")
def device_asm(tmp_path_factory):
    return _compile(tmp_path_factory, "trisolve.hip")


@pytest.fixture(scope="module")
def line_asm(tmp_path_factory):
    return _compile(tmp_path_factory, "linesweep.hip")


def _pk6_kernels(path):
    return sorted(set(re.findall(r"^(_ZN8lssp_amd9k_tri_pk6\w+):", open(path).read(), re.M)))


def test_pk6_instantiations_present(device_asm):
    names = _pk6_kernels(device_asm)
    assert len(names) >= 2, names


def test_pk6_loader_vmcnt_hazard_free(device_asm):
    import check_vmcnt
    for name in _pk6_kernels(device_asm):
        assert check_vmcnt.check_loader(device_asm, name) == 0, name


def test_pk6_no_scratch(device_asm):
    text = open(device_asm).read()
    for name in _pk6_kernels(device_asm):
        m = re.search(r"\.amdhsa_kernel " + name + r"\n(.*?)\.end_amdhsa_kernel", text, re.S)
        assert m, name
        priv = int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", m.group(1)).group(1))
        assert priv == 0, (name, priv)


def test_line2_instantiations_hazard_free_and_no_scratch(line_asm):
    """k_line2 (two levels per step): every instantiation, TRACE included,
    hazard-free on its loaders' / poller's asm-issued DMAs and without scratch."""
    import check_vmcnt
    names = sorted(set(re.findall(r"^(_ZN8lssp_amd7k_line2\w+):", open(line_asm).read(), re.M)))
    assert len(names) >= 4, names
    text = open(line_asm).read()
    for name in names:
        assert check_vmcnt.check_loader(line_asm, name) == 0, name
        m = re.search(r"\.amdhsa_kernel " + name + r"\n(.*?)\.end_amdhsa_kernel", text, re.S)
        assert int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", m.group(1)).group(1)) == 0, name


@pytest.fixture(scope="module")
def fill_asm(tmp_path_factory):
    return _compile(tmp_path_factory, "linefill.hip")


def test_linefill_instantiations_hazard_free_and_no_scratch(fill_asm):
    """k_linef (the 7-point ILU(1) line sweep): every instantiation hazard-free
    on its loaders' / poller's asm-issued DMAs and without scratch."""
    import check_vmcnt
    names = sorted(set(re.findall(r"^(_ZN8lssp_amd7k_linef\w+):", open(fill_asm).read(), re.M)))
    assert len(names) >= 4, names
    text = open(fill_asm).read()
    for name in names:
        assert check_vmcnt.check_loader(fill_asm, name) == 0, name
        m = re.search(r"\.amdhsa_kernel " + name + r"\n(.*?)\.end_amdhsa_kernel", text, re.S)
        assert int(re.search(r"\.amdhsa_private_segment_fixed_size (\d+)", m.group(1)).group(1)) == 0, name
