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

# every printed line is compared; only wall-clock timings differ by nature
TIMED = re.compile(r"time")
NUM = re.compile(r"[-+]?\d+(\.\d*)?([eE][-+]?\d+)?")


def _run(path, log=None, **env):
    e = dict(os.environ, **env)
    out = subprocess.run([path], capture_output=True, text=True, timeout=120, env=e, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    return [NUM.sub("<t>", ln.rstrip()) if TIMED.search(ln) else ln.rstrip() for ln in out.stdout.splitlines()]


def test_exam_binaries_present():
    assert os.path.exists(REF) and os.path.exists(AMD), "run __graft_entry__.build() where /root/reference exists"


def test_exam_drop_in_serial_reduction_prints_what_the_reference_prints():
    ref = _run(REF)
    amd = _run(AMD, LSSP_AMD_REDUCE="serial")
    assert any(ln.startswith("gmres: total iteration: 49") for ln in ref)
    assert amd == ref


def test_exam_drop_in_tree_reduction_converges_alike():
    ref = [ln for ln in _run(REF) if ln.startswith(("gmres: total iteration", "verification"))]
    amd = [ln for ln in _run(AMD) if ln.startswith(("gmres: total iteration", "verification"))]
    nits = lambda lines: int(next(ln for ln in lines if ln.startswith("gmres: total iteration")).split()[-1])
    res = lambda lines: float(next(ln for ln in lines if ln.startswith("verification")).split()[-1])
    assert abs(nits(amd) - nits(ref)) <= 1
    assert res(amd) <= 1e-7 * 100  # ||b|| = 100: the rbn criterion of the run


# ---- every driver through the binding ---------------------------------------
# oracle/drive_solvers.cxx: an exam.cxx-style caller of the reference API
# (lssp_solver_create / set_* / assemble / solve) parameterised by solver, PC
# and grid, linked against the reference alone (drive_ref) and through
# integration/amd_backend.cxx (drive_amd).  In SERIAL reduction mode the two
# print the same nits, residual and x digests, digit for digit.
DRV_REF = os.path.join(ROOT, "oracle", "_ref", "drive_ref")
DRV_AMD = os.path.join(ROOT, "oracle", "_ref", "drive_amd")
ALL_SOLVERS = {"gmres": 0, "lgmres": 1, "gmres_r": 2, "bicgstab": 4, "bicgstabl": 5, "bicgsafe": 6, "cg": 7,
               "cgs": 8, "gpbicg": 9, "cr": 10, "crs": 11, "bicrstab": 12, "bicrsafe": 13, "gpbicr": 14,
               "qmrcgstab": 15, "tfqmr": 16, "orthomin": 17, "idrs": 18}
# (PC, level, N, maxit, param): ILU(0) on 12^3; no PC on 10^3 with a small restart / l / s
DRV_CONFIGS = {"iluk0": ("1", "0", "12", "300", "0"), "none": ("0", "0", "10", "300", "3")}


def _drive(path, args, **env):
    out = subprocess.run([path, *args], capture_output=True, text=True, timeout=120,
                         env=dict(os.environ, **env), cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("nits ")]
    assert len(lines) == 1, out.stdout[-2000:]
    return lines[0]


@pytest.mark.parametrize("cfg", sorted(DRV_CONFIGS))
@pytest.mark.parametrize("solver", sorted(ALL_SOLVERS))
def test_every_driver_drop_in_serial_reduction_bitwise(solver, cfg):
    assert os.path.exists(DRV_REF) and os.path.exists(DRV_AMD), "run __graft_entry__.build() where /root/reference exists"
    args = [str(ALL_SOLVERS[solver]), *DRV_CONFIGS[cfg]]
    ref = _drive(DRV_REF, args)
    amd = _drive(DRV_AMD, args, LSSP_AMD_REDUCE="serial")
    assert amd == ref


@pytest.mark.parametrize("solver,pc", [("bicgstab", "iluk0"), ("gmres", "iluk0"), ("cg", "none")])
def test_binding_keeps_device_state_across_solves_and_follows_reassemble(solver, pc):
    """drive_solvers REPEAT: a second solve after one lssp_solver_assemble (the
    binding reuses the device A, factors and schedules; only x0 and b travel),
    then lssp_solver_assemble with a new matrix (the binding drops its state
    and re-uploads).  Three runs, each bitwise the reference's in SERIAL mode."""
    args = [str(ALL_SOLVERS[solver]), *DRV_CONFIGS[pc], "1"]
    run = lambda path, **env: [ln for ln in subprocess.run([path, *args], capture_output=True, text=True,
                                                           timeout=120, env=dict(os.environ, **env),
                                                           cwd=ROOT).stdout.splitlines() if ln.startswith("nits ")]
    ref = run(DRV_REF)
    amd = run(DRV_AMD, LSSP_AMD_REDUCE="serial")
    assert len(ref) == 3 and amd == ref
    assert ref[0] != ref[2]  # the re-assembled system really differs


@pytest.mark.parametrize("solver,pc,level", [("bicgstab", "3", "0"), ("gmres", "3", "1"), ("cg", "3", "0"),
                                             ("tfqmr", "3", "0"), ("bicgstab", "1", "0"), ("gmres", "2", "0")])
def test_pc_solve_seam_runs_on_the_device(solver, pc, level):
    """The function-pointer PC seam (type-defs.h:103-105, pc.cxx:219-227):
    PC 3 is an LSSP_PC_USER whose assemble calls lssp_pc_iluk_assemble, so
    pc.solve = lssp_pc_ilu_solve -- the binding runs that whole solve on the
    device; then drive_solvers calls pc.solve(&pc, r, x) and pc.solve(&pc, r, b)
    itself, which the wrapped lssp_pc_ilu_solve applies on the device.  Every
    line bitwise the reference's (SERIAL mode); LSSP_AMD_BINDING_STATS shows
    the calls really took the device."""
    args = [str(ALL_SOLVERS[solver]), pc, level, "12", "300", "0", "2"]

    def run(path, **env):
        out = subprocess.run([path, *args], capture_output=True, text=True, timeout=120,
                             env=dict(os.environ, **env), cwd=ROOT)
        assert out.returncode == 0, out.stderr[-2000:]
        return [ln for ln in out.stdout.splitlines() if ln.startswith(("nits ", "pcsolve "))], out.stderr

    ref, _ = run(DRV_REF)
    amd, err = run(DRV_AMD, LSSP_AMD_REDUCE="serial", LSSP_AMD_BINDING_STATS="1")
    assert len(ref) == 3 and amd == ref
    assert "amd: device solves 1, device pc applies 2" in err
