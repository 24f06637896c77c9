"""The drop-in, end to end: the reference's own example/exam.cxx, unchanged,
linked with the reference-side binding integration/amd_backend.cxx (the three
Krylov drivers wrapped onto lssp_amd) runs on the MI355X and
prints what the reference prints (exam_ref: the same program linked against
the reference alone, the checker).  Both binaries are built here by
oracle/Makefile `exam` from the sources under /root/reference and travel to
the GPU box prebuilt (oracle/_ref/, git-ignored).

exam.cxx: 5-pt Laplacian 100x100, GMRES(60) + ILUK(1), b = 1, x0 = 0.
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = os.path.join(ROOT, "oracle", "_ref", "exam_ref")
AMD = os.path.join(ROOT, "oracle", "_ref", "exam_amd")

pytestmark = pytest.mark.gpu

KEEP = re.compile(r"^(gmres: itr|gmres: total iteration|solution L2 norm|verification|CSR:)")


def _run(path, **env):
    e = dict(os.environ, **env)
    out = subprocess.run([path], capture_output=True, text=True, timeout=120, env=e, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    return [ln.rstrip() for ln in out.stdout.splitlines() if KEEP.match(ln)]


def test_exam_binaries_present():
    assert os.path.exists(REF) and os.path.exists(AMD), "run __graft_entry__.build() where /root/reference exists"


def test_exam_drop_in_serial_reduction_prints_what_the_reference_prints():
    ref = _run(REF)
    amd = _run(AMD, LSSP_AMD_REDUCE="serial")
    assert any(ln.startswith("gmres: total iteration: 49") for ln in ref)
    assert amd == ref


def test_exam_drop_in_tree_reduction_converges_alike():
    ref = _run(REF)
    amd = _run(AMD)
    nits = lambda lines: int(next(ln for ln in lines if ln.startswith("gmres: total iteration")).split()[-1])
    res = lambda lines: float(next(ln for ln in lines if ln.startswith("verification")).split()[-1])
    assert abs(nits(amd) - nits(ref)) <= 1
    assert res(amd) <= 1e-7 * 100  # ||b|| = 100: the rbn criterion of the run
