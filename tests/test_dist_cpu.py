"""world_size-2 gloo rehearsal of the multi-GPU decomposition, on the CPU.

Each rank owns a contiguous row block (ceil(n/P) rows, the partition
lssp_amd_mat_upload_dist enforces), multiplies with its rows after fetching
the x entries it needs, applies block-Jacobi ILU(0) on its diagonal block (the
reference's blk_size path, built with bench.local_block exactly as bench.py
does), and forms every dot as the rank-order sum of rank-local canonical tree
partials.  The run must equal, bit for bit, the oracle's single-process
P-rank mode that the GPU ranks are checked against -- which pins the protocol
the RCCL path implements (comm.cpp) independently of the GPU.
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, N, maxit, out):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
        sys.path.insert(0, root)
        from bench import local_block
        A = O.poisson(3, N)
        n = A.n
        blk = (n + world - 1) // world
        r0 = min(rank * blk, n)
        nl = min(blk, n - r0)
        Ap = (A.Ap[r0:r0 + nl + 1] - A.Ap[r0]).astype(np.int32)
        Aj = A.Aj[A.Ap[r0]:A.Ap[r0 + nl]].copy()
        Ax = A.Ax[A.Ap[r0]:A.Ap[r0 + nl]].copy()
        bp, bj, bx = local_block(Ap, Aj, Ax, r0, nl)
        L, U = O.ilu(O.CSR(nl, bp, bj, bx), "iluk", level=0)

        def gather(v):
            parts = [None] * world
            dist.all_gather_object(parts, v)
            return parts

        def gdot(a, b):
            parts = gather(O.dot(a, b, O.TREE))
            t = parts[0]
            for p in parts[1:]:
                t = t + p
            return t

        def spmv(xl):  # halo: the owned slices of every rank, then the local rows
            xf = np.concatenate(gather(xl))
            return O.spmv(0, O.CSR(nl, Ap, Aj, Ax), xf)

        trace = []

        def tdot(a, b):
            v = gdot(a, b)
            trace.append(v)
            return v

        # solver-bicgstab.cxx:10-175 on the rank's slice
        x = np.zeros(nl)
        b = np.ones(nl)
        r = b - spmv(x)
        rh = r.copy()
        trace.append(np.sqrt(gdot(b, b)))
        res = np.sqrt(gdot(r, r))
        trace.append(res)
        tol = max(res * 1e-7, 1e-7, 1e-7 * trace[0])
        rho0 = alpha = omega = 0.0
        p = v = None
        it = 0
        for it in range(maxit):
            rho1 = tdot(r, rh)
            if it == 0:
                p = r.copy()
            else:
                beta = (rho1 * alpha) / (rho0 * omega)
                p = r + beta * (p - omega * v)
            rho0 = rho1
            ph = O.ilu_apply(L, U, p)
            v = spmv(ph)
            alpha = rho1 / tdot(rh, v)
            s = r - alpha * v
            trace.append(np.sqrt(gdot(s, s)))
            sh = O.ilu_apply(L, U, s)
            t = spmv(sh)
            ts, tt = tdot(t, s), tdot(t, t)
            omega = ts / tt
            x = x + alpha * ph + omega * sh
            r = s - omega * t
            res = np.sqrt(gdot(r, r))
            trace.append(res)
            if res <= tol:
                break
        xs = gather(x)
        if rank == 0:
            out.put((it + 1, res, np.array(trace), np.concatenate(xs)))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,N", [(2, 12), (3, 10)])
def test_multirank_bicgstab_equals_oracle_prank_mode(world, N):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, N, 500, q)) for r in range(world)]
    for p in procs:
        p.start()
    nits, res, trace, x = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    A = O.poisson(3, N)
    Lg, Ug = O.ilu(A, "iluk", level=0, blk=(A.n + world - 1) // world)
    o = O.solve(O.BICGSTAB, A, np.ones(A.n), L=Lg, U=Ug, mode=O.TREE, nranks=world, maxit=500)
    assert nits == o.nits
    assert res == o.residual
    assert np.array_equal(trace, o.trace)
    assert np.array_equal(x, o.x)


def test_threaded_block_factors_equal_oracle_blk_mode():
    """tests/test_gpu_dist.py builds config 4's block-Jacobi oracle factors one
    block per thread; they must be O.ilu(A, blk=ceil(n/P)) bit for bit"""
    import numpy as np
    import oracle as O
    from test_gpu_dist import _bj_factors_threaded
    A = O.poisson(3, 20)
    for P in (3, 8):
        L, U = O.ilu(A, "iluk", level=0, blk=(A.n + P - 1) // P)
        L2, U2 = _bj_factors_threaded(A, P)
        for a, b in ((L, L2), (U, U2)):
            assert np.array_equal(a.Ap, b.Ap) and np.array_equal(a.Aj, b.Aj)
            assert np.array_equal(a.Ax.view(np.int64), b.Ax.view(np.int64))
