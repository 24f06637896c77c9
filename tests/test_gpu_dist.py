"""The multi-rank path of the library on the GPU, with several ranks on ONE device.

RCCL refuses two ranks on one GPU, so these tests carry the protocol's
collectives over the host-staged transport (lssp_amd_comm_init_host, hooks
implemented with torch.distributed gloo in lssp_amd.dist).  Everything else
is the production multi-GPU code: lssp_amd_mat_upload_dist's halo plan (built
through the transport), the pack kernel and halo placement before every SpMV,
rank-local canonical tree partials summed in rank order (k_sum_ranks), and
block-Jacobi ILU(0) per rank (pc-iluk.cxx:411-552 with blk = ceil(n/P)).
Results must equal, bit for bit, the oracle's single-process P-rank mode --
the same check tests/test_dist_cpu.py pins on the CPU.
"""
import os
import socket

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, N, maxit, seed, out, solver="bicgstab", mode=1, pc="bj", level=0):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import lssp_amd
        from bench import local_block
        from inputs import uniform
        from lssp_amd.dist import GlooTransport
        dev = lssp_amd.Device(0, reduction=mode)
        dev.comm_init_host(world, rank, GlooTransport())
        n = N ** 3
        blk = (n + world - 1) // world
        r0 = min(rank * blk, n)
        nl = min(blk, n - r0)
        Ap, Aj, Ax = lssp_amd.poisson(3, N, r0, nl)
        A = lssp_amd.DMat(dev, Ap, Aj, Ax, dist=(n, r0))
        if pc == "global":  # every rank holds the ILU(0) of the WHOLE matrix (pc-iluk.cxx:574)
            gp, gj, gx = lssp_amd.poisson(3, N)
            M = lssp_amd.DILU.create(dev, gp, gj, gx, kind=lssp_amd.ILUK, level=0)
        else:
            bp, bj, bx = local_block(Ap, Aj, Ax, r0, nl)
            M = lssp_amd.DILU.create(dev, bp, bj, bx, kind=lssp_amd.ILUK, level=level)
            if level == 1 and nl % (N * N) == 0:  # a whole-plane slab: the ILU(1) line sweeps
                assert M.sweep_layout()[0] == 2
        # SpMV with a halo: y = A x for a seeded global x
        xg = uniform(seed, n)
        xv = dev.vec(A.nx, np.concatenate([xg[r0:r0 + nl], np.zeros(A.nhalo)]))
        yv = dev.vec(A.nx)
        A.mv_mxy(xv, yv)
        y = yv.download(nl)
        # b = 1, x0 = 0, tree reductions; block-Jacobi ILU(0) except for CG (PC_NON)
        x = dev.vec(A.nx, np.zeros(A.nx))
        b = dev.vec(A.nx, np.ones(A.nx))
        sol = {"bicgstab": lssp_amd.BICGSTAB, "gmres": lssp_amd.GMRES, "cg": lssp_amd.CG,
               "idrs": lssp_amd.IDRS, "bicgstabl": lssp_amd.BICGSTABL}[solver]
        r = lssp_amd.solve(dev, A, None if solver == "cg" else M, x, b, solver=sol, maxit=maxit, restart=30,
                           trace_cap=100000)
        xl = x.download(nl)
        dev.barrier()
        parts = [None] * world
        dist.all_gather_object(parts, (y, xl))
        if rank == 0:
            out.put((r.nits, r.residual, r.trace, np.concatenate([p[0] for p in parts]),
                     np.concatenate([p[1] for p in parts])))
        dev.close()
    finally:
        dist.destroy_process_group()


def _run(world, N, solver, mode, maxit=500, pc="bj", level=0):
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, maxit, 0x5EED, q, solver, mode, pc, level))
             for r in range(world)]
    for p in procs:
        p.start()
    try:
        res = q.get(timeout=150)
    finally:
        for p in procs:
            p.join(timeout=30)
    assert all(p.exitcode == 0 for p in procs)
    return res


@pytest.mark.parametrize("mode", [O.TREE, O.SERIAL], ids=["tree", "serial"])
def test_config4_partition_8_ranks(mode):
    """Config 4's decomposition (8 row blocks = 8 z-slabs, block-Jacobi ILU(0)
    per rank, halo planes, rank-combined dots) with 8 ranks on one GPU at 64^3.
    TREE: bitwise the oracle's 8-rank mode.  SERIAL: the ranks continue each
    other's running sums, so every dot is the reference's sequential sum and
    the run is bitwise the REFERENCE's own block-Jacobi (nblk = 8) solve
    (tests/golden/large.json, from oracle/_ref/libref.so)."""
    import json
    world, N = 8, 64
    nits, res, trace, y, x = _run(world, N, "bicgstab", mode, maxit=5000)
    A = O.poisson(3, N)
    L, U = O.ilu(A, "iluk", level=0, blk=(A.n + world - 1) // world)
    o = O.solve(O.BICGSTAB, A, np.ones(A.n), L=L, U=U, mode=mode, nranks=world, maxit=5000)
    assert nits == o.nits
    assert res == o.residual
    assert np.array_equal(trace, o.trace)
    assert np.array_equal(x, o.x)
    if mode == O.SERIAL:
        from inputs import digest
        with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "large.json")) as f:
            g = [c for c in json.load(f)["cases"] if c["pc"] == {"kind": "bj", "nblk": 8} and c["N"] == N][0]
        assert nits == g["nits"]
        assert res.hex() == g["residual"]
        assert [v.hex() for v in trace] == g["trace"]
        assert digest(x) == g["x_sha256"]


def _c4_worker(rank, world, port, out):
    """one rank of config 4 at full size: its 512^3 / 8 z-slab, block-Jacobi ILU(0)"""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import lssp_amd
        from bench import local_block
        from inputs import digest
        from lssp_amd.dist import GlooTransport
        dev = lssp_amd.Device(0, reduction=lssp_amd.TREE)
        dev.comm_init_host(world, rank, GlooTransport())
        N = 512
        n = N ** 3
        blk = (n + world - 1) // world
        r0 = min(rank * blk, n)
        nl = min(blk, n - r0)
        Ap, Aj, Ax = lssp_amd.poisson(3, N, r0, nl)
        A = lssp_amd.DMat(dev, Ap, Aj, Ax, dist=(n, r0))
        bp, bj, bx = local_block(Ap, Aj, Ax, r0, nl)
        del Ap, Aj, Ax
        M = lssp_amd.DILU.create(dev, bp, bj, bx, kind=lssp_amd.ILUK, level=0)
        del bp, bj, bx
        layout = M.sweep_layout()
        b = dev.vec(A.nx, np.ones(A.nx))
        x = dev.vec(A.nx, np.zeros(A.nx))
        # (1) the first three iterations, zero tolerances: trace and x
        r3 = lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0,
                            maxit=3, trace_cap=64)
        x3 = digest(x.download(nl))
        # (2) converged at the reference's default tolerances
        x.upload(np.zeros(A.nx))
        rc = lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, maxit=5000)
        z = dev.vec(A.nx)
        A.mv_amxpbyz(-1.0, x, 1.0, b, z)  # b - A x with this rank's halo
        zh = z.download(nl)
        ss = float(np.dot(zh, zh))
        dev.barrier()
        parts = [None] * world
        dist.all_gather_object(parts, (x3, ss, layout))
        if rank == 0:
            out.put((r3.nits, r3.residual, r3.trace, [p[0] for p in parts], rc.nits, rc.residual,
                     sum(p[1] for p in parts), [p[2] for p in parts]))
        dev.close()
    finally:
        dist.destroy_process_group()


def _bj_factors_threaded(A, nblk):
    """the oracle's block-Jacobi ILU(0) factors (O.ilu(A, blk=ceil(n/nblk))) built
    block by block on nblk threads (ctypes drops the GIL): each block's factor is
    the ILU(0) of its diagonal block (pc-iluk.cxx:441-535), columns shifted back"""
    from concurrent.futures import ThreadPoolExecutor
    from bench import local_block
    n = A.n
    blk = (n + nblk - 1) // nblk

    def one(q):
        r0 = q * blk
        nl = min(blk, n - r0)
        e0, e1 = int(A.Ap[r0]), int(A.Ap[r0 + nl])
        bp, bj, bx = local_block(A.Ap[r0:r0 + nl + 1] - e0, A.Aj[e0:e1], A.Ax[e0:e1], r0, nl)
        return O.ilu(O.CSR(nl, bp, bj, bx), "iluk", level=0)

    with ThreadPoolExecutor(nblk) as ex:
        parts = list(ex.map(one, range((n + blk - 1) // blk)))

    def cat(fs):
        ap, off = [np.zeros(1, np.int64)], 0
        for f in fs:
            ap.append(f.Ap[1:].astype(np.int64) + off)
            off += int(f.Ap[-1])
        return O.CSR(n, np.concatenate(ap).astype(np.int32),
                     np.concatenate([f.Aj + q * blk for q, f in enumerate(fs)]).astype(np.int32),
                     np.concatenate([f.Ax for f in fs]))

    return cat([p[0] for p in parts]), cat([p[1] for p in parts])


@pytest.mark.timeout(900)
def test_config4_full_size_8_ranks_on_one_gpu():
    """Config 4 at its FULL size: 7-pt 512^3 (n = 134,217,728) over 8 ranks --
    8 z-slabs of 64 planes, block-Jacobi ILU(0) per rank on the line sweeps
    (pc-iluk.cxx:411-552 with blk = n / 8), halo planes and rank-combined dots
    over the host transport, all 8 ranks on this one GPU.  The first three
    BiCGSTAB iterations (every traced scalar, each rank's x) are bitwise the
    oracle's 8-rank TREE mode on the whole 512^3 system, computed here while
    the ranks run; then the solve converges at the reference's default
    tolerances (lssp.cxx:11-13) below the stop scale, and the recomputed global
    true residual ||b - A x|| is within 2x that scale."""
    import math
    import torch.multiprocessing as mp
    from inputs import digest
    world, N = 8, 512
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c4_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        # the oracle's 8-rank mode on the whole system, concurrently with the ranks
        A = O.poisson(3, N)
        n = A.n
        blk = (n + world - 1) // world
        L, U = _bj_factors_threaded(A, world)  # == O.ilu(A, "iluk", level=0, blk=blk), one block per thread
        o = O.solve(O.BICGSTAB, A, np.ones(n), L=L, U=U, rtol=0.0, atol=0.0, rbtol=0.0, maxit=3, mode=O.TREE,
                    nranks=world, trace_cap=64)
        del L, U, A
        want_x = [digest(o.x[q0:q0 + blk]) for q0 in range(0, n, blk)]
        nits3, res3, trace3, x3, nits, res, ss, layouts = q.get(timeout=800)
    finally:
        for p in procs:
            p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(lay[0] == 1 for lay in layouts), layouts  # every slab on the ILU(0) line sweeps
    assert nits3 == o.nits == 3
    assert res3 == o.residual
    assert np.array_equal(trace3.view(np.int64), o.trace.view(np.int64))
    assert x3 == want_x
    scale = 1e-7 * math.sqrt(n)  # max(rtol ||r0||, atol, rb ||b||), r0 = b = 1
    true_res = math.sqrt(ss)
    print(f"\nconfig 4, 8 ranks: {nits} iterations, residual {res:.6e}, true residual {true_res:.6e}, "
          f"stop scale {scale:.6e}")
    assert 0 < nits < 5000 and res <= scale
    assert true_res <= 2.0 * scale


@pytest.mark.parametrize("world,N,solver", [(2, 12, "bicgstab"), (3, 10, "bicgstab"), (4, 16, "bicgstab"),
                                             (2, 12, "gmres"), (3, 11, "gmres"), (2, 12, "cg"), (4, 13, "cg"),
                                             # IDR(4): each rank keeps its rows of the global rand() shadow space
                                             (2, 12, "idrs"), (3, 10, "bicgstabl")])
def test_multirank_on_one_gpu_equals_oracle_prank_mode(world, N, solver):
    nits, res, trace, y, x = _run(world, N, solver, O.TREE)
    from inputs import uniform
    A = O.poisson(3, N)
    assert np.array_equal(y, O.spmv(0, A, uniform(0x5EED, A.n)))
    L = U = None
    if solver != "cg":
        L, U = O.ilu(A, "iluk", level=0, blk=(A.n + world - 1) // world)
    sol = {"bicgstab": O.BICGSTAB, "gmres": O.GMRES, "cg": O.CG, "idrs": O.IDRS, "bicgstabl": O.BICGSTABL}[solver]
    o = O.solve(sol, A, np.ones(A.n), L=L, U=U, mode=O.TREE, nranks=world, maxit=500,
                restart=4 if solver in ("idrs", "bicgstabl") else 30)  # l / s = 4, the library default
    assert nits == o.nits
    assert res == o.residual
    assert np.array_equal(trace, o.trace)
    assert np.array_equal(x, o.x)


@pytest.mark.parametrize("tail", ["default", "2"], ids=["tail-default", "tail-forced"])
@pytest.mark.parametrize("world,N", [(2, 16), (4, 16)])
def test_multirank_ilu1_line_sweeps_equal_oracle_prank_mode(world, N, tail, monkeypatch):
    """block-Jacobi ILU(1) (the reference's default level) per rank: each whole-plane
    slab's factor runs on the skewed line sweeps; BiCGSTAB in tree order equals the
    oracle's P-rank mode bit for bit.  LSSP_AMD_TAIL=2 (inherited by the spawned
    ranks) makes an ineligible tail product fail instead of falling back, so the
    forced case proves the distributed tail (halo-free chunks in the U sweep, then
    spmv_boundary) ran."""
    if tail != "default":
        monkeypatch.setenv("LSSP_AMD_TAIL", tail)
    nits, res, trace, y, x = _run(world, N, "bicgstab", O.TREE, level=1)
    A = O.poisson(3, N)
    L, U = O.ilu(A, "iluk", level=1, blk=(A.n + world - 1) // world)
    o = O.solve(O.BICGSTAB, A, np.ones(A.n), L=L, U=U, mode=O.TREE, nranks=world, maxit=500, restart=30)
    assert nits == o.nits
    assert res == o.residual
    assert np.array_equal(trace, o.trace)
    assert np.array_equal(x, o.x)


def _bad_worker(rank, world, port, bad_rank, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import lssp_amd
        from lssp_amd.dist import GlooTransport
        dev = lssp_amd.Device(0)
        dev.comm_init_host(world, rank, GlooTransport())
        N = 8
        n = N ** 3
        blk = (n + world - 1) // world
        r0 = min(rank * blk, n)
        nl = min(blk, n - r0)
        Ap, Aj, Ax = lssp_amd.poisson(3, N, r0, nl)
        if rank == bad_rank:
            Aj = Aj.copy()
            Aj[3] = n + 7  # a column outside the global matrix
        try:
            lssp_amd.DMat(dev, Ap, Aj, Ax, dist=(n, r0))
            status = 0
        except lssp_amd.LsspError as e:
            status = e.status
        out.put((rank, status))
        dev.close()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("bad_rank", [0, 1])
def test_dist_upload_bad_input_fails_on_every_rank(bad_rank):
    """lssp_amd_mat_upload_dist agrees on the input checks before any
    collective: one rank's bad column makes BOTH ranks return EINVAL instead
    of leaving the good one waiting in the halo-plan exchange."""
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bad_worker, args=(r, 2, port, bad_rank, q)) for r in range(2)]
    for p in procs:
        p.start()
    try:
        got = dict(q.get(timeout=120) for _ in range(2))
    finally:
        for p in procs:
            p.join(timeout=30)
    assert got == {0: 1, 1: 1}
    assert all(p.exitcode == 0 for p in procs)


def test_rccl_one_rank_transport_selftest():
    """The RCCL branch of the transport on one GPU: a real 1-rank communicator
    (lssp_amd_comm_init with nranks = 1), then lssp_amd_comm_selftest drives
    ncclAllGather and a grouped ncclSend/ncclRecv round to itself on the
    communication stream between the same two events spmv_halo uses, and
    checks every word.  A single-rank solve on the same context afterwards is
    still bitwise the oracle (the communicator does not change its path)."""
    import lssp_amd
    dev = lssp_amd.Device(0)
    try:
        dev.comm_init(1, 0, lssp_amd.comm_unique_id())
        dev.comm_selftest()
        dev.comm_selftest()  # the events and comm stream are reusable
        A = O.poisson(3, 16)
        Ad = lssp_amd.DMat(dev, A.Ap, A.Aj, A.Ax)
        x, b = dev.vec(A.n, np.zeros(A.n)), dev.vec(A.n, np.ones(A.n))
        r = lssp_amd.solve(dev, Ad, None, x, b, solver=lssp_amd.CG, maxit=30, trace_cap=256)
        o = O.solve(O.CG, A, np.ones(A.n), maxit=30, mode=O.TREE)
        assert r.nits == o.nits and np.array_equal(r.trace, o.trace) and np.array_equal(x.download(), o.x)
    finally:
        dev.close()


@pytest.mark.parametrize("world,N,mode", [(2, 32, O.SERIAL), (3, 20, O.SERIAL), (4, 16, O.TREE), (2, 24, O.TREE)],
                         ids=["2r32-serial", "3r20-serial", "4r16-tree", "2r24-tree"])
def test_global_ilu_on_p_ranks(world, N, mode):
    """The reference's own preconditioner on P ranks: every rank holds the
    ILU(0) factors of the whole matrix (pc-iluk.cxx:574, blk_size = n) and an
    apply all-gathers the rhs blocks, sweeps the global system and keeps the
    rank's rows.  SERIAL: the ranks continue each other's running sums, so the
    run is bitwise the single-process reference order -- the same iteration
    count as one GPU, unlike block-Jacobi.  TREE: bitwise the oracle's P-rank
    reduction order with the global factors."""
    nits, res, trace, y, x = _run(world, N, "bicgstab", mode, maxit=5000, pc="global")
    A = O.poisson(3, N)
    L, U = O.ilu(A, "iluk", level=0)
    o = O.solve(O.BICGSTAB, A, np.ones(A.n), L=L, U=U, mode=mode, nranks=1 if mode == O.SERIAL else world,
                maxit=5000)
    assert nits == o.nits
    assert res == o.residual
    assert np.array_equal(trace, o.trace)
    assert np.array_equal(x, o.x)
    if mode == O.SERIAL and N == 32:  # the reference takes 21 iterations at 32^3
        assert nits == 21


def test_bench_gpus_2_launches_two_ranks():
    """`python bench.py --gpus 2` run plainly starts two ranks itself (here on
    one device over the host transport, --share-gpu) and reports n_gpus 2 and a
    2-rank communicator -- the driver's multi-GPU scaling run cannot silently
    measure one rank."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--share-gpu", "--grid", "32",
                        "--steps", "5", "--warmup", "1", "--no-cpu", "--spmv-reps", "3", "--apply-reps", "2",
                        "--config4-steps", "0"],
                       env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["config"]["comm_ranks"] == 2 and line["steps"] == 5
