#!/usr/bin/env python3
"""Benchmark of the LSSP Krylov hot path on MI355X (BASELINE.json metric).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--grid 216|256|512]

--gpus N > 1 run directly starts N ranks (torch.distributed.run, one process
per GPU, 127.0.0.1 rendezvous); under an external launcher WORLD_SIZE must
equal N.  --grid 512 is config 4's matrix (134 M rows; 512^3 over 8 GPUs).

Workload: 7-point Poisson on a 216^3 grid (n = 10,077,696 rows, 70,263,936
nnz -- the "n=10M" of BASELINE.json), fp64, b = 1, x0 = 0, BiCGSTAB with an
ILUK(0) preconditioner (solver-bicgstab.cxx, pc-iluk.cxx).  One STEP is one
BiCGSTAB iteration: 2 SpMV, 2 ILU applies (4 triangular sweeps), 4 dots and
2 norms.  The solve runs with zero tolerances, so it performs exactly the
requested number of iterations.  value = iterations per second of the whole
job.  With N > 1 (torchrun, one process per GPU) the same global matrix is
row-partitioned into N z-slabs (strong scaling); halos move with RCCL
send/recv and dots with an RCCL all-gather; the preconditioner becomes
block-Jacobi ILU(0) per slab (the reference's blk_size path).

The roofline object describes the dominant operator, the ILU(0) apply
(pc.solve: the rhs gather and the two line sweeps k_line2, L then U --
rocprof attributes ~65% of a step to them); roofline_spmv describes the
metric's SpMV kernel, y = A x
(lssp_mv_mxy).  Both are timed live with HIP events on the library's stream.
traffic: HBM bytes per launch from rocprofv3 PMC counters (FETCH_SIZE x 2 on
gfx950, + WRITE_SIZE), read from profiles/pmc_traffic.json when present.
config4: the same BiCGSTAB + ILU(0) step on config 4's 7-pt 512^3 matrix
(134 M rows) over the same N ranks -- z-slabs, block-Jacobi ILU(0) per rank
on N > 1 -- timed the same way (>= 10 iterations, barrier + sync, max over
ranks), so the driver's N = 1, 2, 4, 8 runs record BASELINE.md 3's curve on
the matrix it names; --config4-steps 0 skips it.  The headline value stays on
216^3.
cpu_baseline is the REFERENCE itself (oracle/_ref/libref.so, compiled from
/root/reference, g++ -O2, 1 core) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def spmv_bytes(nnz: int, n: int, coded: bool = False) -> int:
    """algorithmic bytes of y = A x: Ax 8 + Aj 4 per nnz, Ap 4 + x 8 + y 8 per row.
    coded: the device layout's 1-byte diagonal id replaces Aj's 4 bytes
    (lssp_amd_mat_layout; 7-pt: 7 offsets), so the kernel moves 9 per nnz"""
    return (9 if coded else 12) * nnz + 20 * n + 4


def ilu_apply_bytes(nnzL: int, nnzU: int, n: int) -> int:
    """SURVEY 8(d) B_ilu = 12 (nnzL_strict + nnzU) + 40 n: the strict L entries
    and all of U (8 + 4 per entry; L's unit diagonal is not stored), row
    pointers, rhs read, the L sweep's output written and read back by the U
    sweep, x written.  nnzL counts L's unit diagonal (one per row)."""
    return 12 * (nnzL - n + nnzU) + 40 * n


def pmc_traffic(kernel: str):
    """HBM bytes per launch measured with rocprofv3 --pmc (tools/pmc_traffic.py)"""
    try:
        with open(os.path.join(HERE, "profiles", "pmc_traffic.json")) as f:
            return json.load(f).get(kernel)
    except (OSError, ValueError):
        return None


def build_local(N: int, rank: int, P: int):
    import lssp_amd
    n = N ** 3
    blk = (n + P - 1) // P
    row0 = min(rank * blk, n)
    nl = min(blk, n - row0)
    Ap, Aj, Ax = lssp_amd.poisson(3, N, row0, nl)
    return n, row0, nl, Ap, Aj, Ax


def local_block(Ap, Aj, Ax, row0, nl):
    """the rank's diagonal block (block-Jacobi, pc-iluk.cxx:441-447)"""
    keep = (Aj >= row0) & (Aj < row0 + nl)
    rows = np.repeat(np.arange(nl), np.diff(Ap))
    cnt = np.bincount(rows[keep], minlength=nl)
    bp = np.zeros(nl + 1, np.int32)
    np.cumsum(cnt, out=bp[1:])
    return bp, (Aj[keep] - row0).astype(np.int32), Ax[keep]


def cpu_baseline(N: int, iters: int):
    """The reference on a bounded sample: SpMV reps + BiCGSTAB+ILU(0) iterations."""
    import oracle as O
    if not O.ref_available():
        return None
    A = O.poisson(3, N)
    x = np.random.default_rng(0).uniform(-1, 1, A.n)
    z = np.zeros(A.n)
    R = O.ref()
    O.ref_spmv(0, A, x, z=z)
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        O.ref_spmv(0, A, x, z=z)
    t_spmv = (time.perf_counter() - t0) / reps
    b = np.ones(A.n)
    r = O.ref_solve(O.BICGSTAB, A, b, pc=O.PC_ILUK, level=0, rtol=0.0, atol=0.0, rbtol=0.0, maxit=iters,
                    trace_cap=16)
    del R
    cpu = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            cpu = next(line.split(":", 1)[1].strip() for line in f if line.startswith("model name"))
    except Exception:
        pass
    return {"value": round(r.nits / r.t_solve, 4), "unit": "iters/s", "cores": 1, "kind": "reference",
            "sample": f"reference lssp_solver_solve BiCGSTAB+ILUK(0) on the same 7-pt {N}^3 system, "
                      f"{r.nits} iterations in {r.t_solve:.2f} s (ILU setup {r.t_setup:.2f} s, not counted); "
                      f"lssp_mv_mxy {t_spmv * 1e3:.1f} ms = {spmv_bytes(A.nnz, A.n) / t_spmv / 1e9:.2f} GB/s",
            "spmv_gbps": round(spmv_bytes(A.nnz, A.n) / t_spmv / 1e9, 3),
            "cpu_model": cpu, "host_cpus": os.cpu_count()}


def measure_hbm_peak(dev, stream, gpu, e0, e1):
    """Measured HBM peaks beside the 8 TB/s spec ("also record a
    measured copy-kernel peak"), 2^27 doubles (1 GiB), bytes over HIP-event
    time on the library's stream: "read" = lssp_amd_stream_read (k_read16: every
    word once by 16-byte non-temporal loads, 8 in flight per lane -- the
    streaming-read ceiling the SpMV and the sweeps are compared with), "copy" =
    the library's vec_copy (k_copy16).  An auxiliary number: a failure here is
    reported in the detail and never costs the bench line."""
    import torch

    try:
        nc = 1 << 27
        src = torch.empty(nc, dtype=torch.float64, device=f"cuda:{gpu}").uniform_(-1, 1)
        dst = torch.empty_like(src)
        sink = torch.zeros(2, dtype=torch.float64, device=src.device)
        torch.cuda.synchronize()
        best = {}
        for how in ("read", "copy"):
            def op():
                if how == "read":
                    st = dev.L.lssp_amd_stream_read(dev.h, src.data_ptr(), nc, sink.data_ptr())
                else:
                    st = dev.L.lssp_amd_vec_copy(dev.h, dst.data_ptr(), src.data_ptr(), nc)
                assert st == 0, st
            for _ in range(3):
                op()
            times = []
            for _ in range(5):
                e0.record(stream)
                for _ in range(10):
                    op()
                e1.record(stream)
                e1.synchronize()
                times.append(e0.elapsed_time(e1) / 10 * 1e-3)
            nbytes = 8.0 * nc * (1 if how == "read" else 2)
            best[how] = round(nbytes / min(times) / 1e9, 1)
        # the fold is checkable: XOR of all 64-bit words
        w = src.view(torch.int64)
        want = int(np.bitwise_xor.reduce(w.cpu().numpy()))
        got = int(sink.view(torch.int64)[0].item())
        best["read_checked"] = got == want
        # the read kernel's number only when its fold checked out; else the copy peak
        peak_measured = best["read"] if best["read_checked"] else best["copy"]
        del src, dst
        return peak_measured, best
    except Exception as ex:  # noqa: BLE001
        return None, {"error": repr(ex)[:200]}


def config4_leg(dev, rank: int, world: int, steps: int, warmup: int = 2):
    """Config 4 (BASELINE.json configs[3]): 7-pt Poisson 512^3 (n = 134,217,728),
    BiCGSTAB + ILU(0), row-partitioned over the same N ranks as the headline
    (z-slabs, block-Jacobi ILU(0) per rank -- the reference's blk_size path,
    pc-iluk.cxx:411-552 -- halos and dots over RCCL; one rank: the global
    ILU(0)).  Timed like the headline: barrier + device sync on both sides, the
    max over ranks.  Its it/s at N = 1, 2, 4, 8 is the curve BASELINE.md 3 asks
    for; the headline value stays on 216^3."""
    import torch
    import torch.distributed as dist
    import lssp_amd
    N = 512
    t0 = time.perf_counter()
    n, row0, nl, Ap, Aj, Ax = build_local(N, rank, world)
    if world > 1:
        A = lssp_amd.DMat(dev, Ap, Aj, Ax, dist=(n, row0))
        bp, bj, bx = local_block(Ap, Aj, Ax, row0, nl)
        del Ap, Aj, Ax
        M = lssp_amd.DILU.create(dev, bp, bj, bx, kind=lssp_amd.ILUK, level=0)
        del bp, bj, bx
    else:
        A = lssp_amd.DMat(dev, Ap, Aj, Ax)
        M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=0)
        del Ap, Aj, Ax
    x = dev.vec(A.nx, np.zeros(A.nx))
    b = dev.vec(A.nx, np.ones(A.nx))
    setup_s = time.perf_counter() - t0

    def run(iters):
        return lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0,
                              maxit=iters)

    if warmup > 0:
        run(warmup)
    if world > 1:
        dist.barrier()
    dev.sync()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    res = run(steps)
    dev.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t1
    if world > 1:
        t = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    assert res.nits == steps, f"config4: expected {steps} iterations, got {res.nits}"
    out = {"workload": f"7-pt Poisson {N}^3 (n={n}, nnz={7 * N ** 3 - 6 * N ** 2}), BiCGSTAB + ILUK(0)"
                       f"{' block-Jacobi per rank' if world > 1 else ''}, b=1, x0=0, fp64",
           "value": round(steps / el, 3), "unit": "iters/s", "ms_per_step": round(el / steps * 1e3, 4),
           "steps": steps, "warmup": warmup, "n_gpus": world, "rows_per_rank": nl,
           "partition": f"{world} z-slab row blocks", "levels_per_sweep": M.levelsL,
           "comm_ranks": dev.comm_nranks() if world > 1 else 1, "setup_s": round(setup_s, 2)}
    for o in (x, b, M, A):
        o.close()
    return out


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n: int) -> int:
    """python -m torch.distributed.run --nproc-per-node n bench.py <same args>,
    rendezvous on 127.0.0.1; returns the launcher's exit code."""
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC only on this host driver
    env.setdefault("OMP_NUM_THREADS", "4")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--grid", type=int, default=216)
    ap.add_argument("--spmv-reps", type=int, default=50)
    ap.add_argument("--apply-reps", type=int, default=10)
    ap.add_argument("--cpu-iters", type=int, default=8)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--config4-steps", type=int, default=10,
                    help="BiCGSTAB iterations timed on config 4's 512^3 matrix over the same N ranks (0: skip)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="rehearsal: every rank on device 0, collectives over the host-staged gloo transport "
                         "(RCCL refuses two ranks on one GPU); not a scaling measurement")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        # one process per GPU: start the N ranks under torch.distributed.run as a
        # child (nothing has touched the GPU in this process) and exit with its code
        sys.exit(launch_ranks(args.gpus))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}")
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import torch
    import torch.distributed as dist
    if world > 1:
        dist.init_process_group("gloo")  # control plane only; the data path is RCCL in the library
    gpu = 0 if args.share_gpu else local_rank
    torch.cuda.set_device(gpu)

    import lssp_amd
    dev = lssp_amd.Device(gpu)
    if world > 1 and args.share_gpu:
        from lssp_amd.dist import GlooTransport
        dev.comm_init_host(world, rank, GlooTransport())
    elif world > 1:
        uid = [lssp_amd.comm_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(uid, src=0)
        dev.comm_init(world, rank, uid[0])

    N = args.grid
    t_setup0 = time.perf_counter()
    n, row0, nl, Ap, Aj, Ax = build_local(N, rank, world)
    if world > 1:
        A = lssp_amd.DMat(dev, Ap, Aj, Ax, dist=(n, row0))
        bp, bj, bx = local_block(Ap, Aj, Ax, row0, nl)
        M = lssp_amd.DILU.create(dev, bp, bj, bx, kind=lssp_amd.ILUK, level=0)
    else:
        A = lssp_amd.DMat(dev, Ap, Aj, Ax)
        M = lssp_amd.DILU.create(dev, Ap, Aj, Ax, kind=lssp_amd.ILUK, level=0)
    nnz_local = int(Ap[-1])
    x = dev.vec(A.nx, np.zeros(A.nx))
    b = dev.vec(A.nx, np.ones(A.nx))
    y = dev.vec(A.nx)
    t_setup = time.perf_counter() - t_setup0

    comm_ranks = dev.comm_nranks() if world > 1 else 1
    if comm_ranks != world:
        raise SystemExit(f"bench.py: the communicator has {comm_ranks} ranks, WORLD_SIZE={world}")

    # ---- SpMV roofline leg: y = A x, HIP events on the library's stream ----
    xs = dev.vec(A.nx, np.random.default_rng(rank).uniform(-1, 1, A.nx))
    stream = torch.cuda.ExternalStream(dev.stream)
    for _ in range(5):
        A.mv_mxy(xs, y)
    dev.sync()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(args.spmv_reps):
        A.mv_mxy(xs, y)
    e1.record(stream)
    e1.synchronize()
    spmv_ms = e0.elapsed_time(e1) / args.spmv_reps
    ndiag = A.ndiag
    spmv_b = spmv_bytes(nnz_local, nl, coded=ndiag > 0)
    spmv_gbs = spmv_b / (spmv_ms * 1e-3) / 1e9
    csr_equiv_gbs = spmv_bytes(nnz_local, nl) / (spmv_ms * 1e-3) / 1e9

    # ---- ILU apply roofline leg (the dominant operator): applies enqueued back
    # to back (lssp_amd_ilu_apply_async; the synchronous C-ABI apply adds a host
    # round trip per call that a solve's queued applies do not pay) ----
    zs = dev.vec(A.nx)
    for _ in range(3):
        M.apply(zs, xs)
    e0.record(stream)
    for _ in range(args.apply_reps):
        M.apply_async(zs, xs)
    e1.record(stream)
    e1.synchronize()
    M.check()
    apply_ms = e0.elapsed_time(e1) / args.apply_reps
    apply_b = ilu_apply_bytes(M.nnzL, M.nnzU, nl)
    apply_gbs = apply_b / (apply_ms * 1e-3) / 1e9

    # ---- measured HBM copy / read peak (rank 0) ----
    peak_measured, peak_detail = None, None
    if rank == 0:
        peak_measured, peak_detail = measure_hbm_peak(dev, stream, gpu, e0, e1)

    # ---- BiCGSTAB steps ----
    def run(iters):
        return lssp_amd.solve(dev, A, M, x, b, solver=lssp_amd.BICGSTAB, tol_rel=0.0, tol_abs=0.0, tol_rb=0.0,
                              maxit=iters)

    if args.warmup > 0:
        run(args.warmup)
    if world > 1:
        dist.barrier()
    dev.sync()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    res = run(args.steps)
    dev.sync()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        g = torch.tensor([spmv_gbs], dtype=torch.float64)
        dist.all_reduce(g, op=dist.ReduceOp.SUM)
        spmv_gbs_total = float(g.item())
    else:
        spmv_gbs_total = spmv_gbs
    assert res.nits == args.steps, f"expected {args.steps} iterations, got {res.nits}"

    if rank == 0:
        it_s = args.steps / elapsed
        out = {
            "metric": "fp64 CSR SpMV GB/s (% HBM peak) + BiCGSTAB iters/s, 7-pt Poisson n=10M",
            "value": round(it_s, 3),
            "unit": "iters/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 4),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": f"7-pt Poisson {N}^3 (n={n}, nnz={int(7 * N ** 3 - 6 * N ** 2)}), "
                                   f"BiCGSTAB + ILUK(0){' block-Jacobi per rank' if world > 1 else ''}, "
                                   "b=1, x0=0, fp64 CSR int32",
                       "rows": n, "partition": f"{world} z-slab row blocks", "reduction": "tree",
                       "transport": ("host-staged gloo, all ranks on GPU 0 (rehearsal, not a scaling number)"
                                     if args.share_gpu and world > 1 else "rccl" if world > 1 else "none"),
                       "comm_ranks": comm_ranks},
            "spmv": {"gbps": round(spmv_gbs_total, 1), "frac_hbm_peak": round(spmv_gbs / HBM_PEAK_GBS, 4),
                     "ms_per_call": round(spmv_ms, 5),
                     "column_stream": (f"1-byte diagonal ids ({ndiag} offsets)" if ndiag else "int32 columns"),
                     "csr_int32_equivalent_gbps": round(csr_equiv_gbs, 1)},
            "roofline": {"bound": "hbm", "achieved": round(apply_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(apply_gbs / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("ilu_apply"),
                         "kernel": "ILU(0) apply = k_line_rhs (rhs -> the L sweep's stream) + k_line2 (L sweep "
                                   "-> the U sweep's rhs stream) + k_line2 (U sweep -> x in natural order); "
                                   f"latency-bound: 2 x {M.levelsL} dependent levels, two per workgroup step",
                         "bytes_per_launch": apply_b, "ms_per_launch": round(apply_ms, 5),
                         "peak_measured": peak_measured, "peak_measured_detail": peak_detail,
                         "frac_of_measured_peak": round(apply_gbs / peak_measured, 4) if peak_measured else None},
            "roofline_spmv": {"bound": "hbm", "achieved": round(spmv_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                              "frac": round(spmv_gbs / HBM_PEAK_GBS, 4), "traffic": pmc_traffic("k_spmv3"),
                              "kernel": f"k_spmv3<EPI_MXY,0,{'true' if ndiag else 'false'}> (y = A x)",
                              "bytes_per_launch": spmv_b, "ms_per_launch": round(spmv_ms, 5),
                              "peak_measured": peak_measured,
                              "frac_of_measured_peak": round(spmv_gbs / peak_measured, 4) if peak_measured else None},
            "ilu": {"levels_L": M.levelsL, "levels_U": M.levelsU, "setup_s": round(M.setup_seconds, 3)},
            "setup_s": round(t_setup, 2),
        }
    # ---- config 4 (512^3 over the same ranks): the scaling curve's matrix ----
    if N == 512:
        args.config4_steps = 0  # the headline is config 4's matrix already
    if args.config4_steps > 0:
        for o in (x, b, y, xs, zs, M, A):
            o.close()
        c4 = config4_leg(dev, rank, world, args.config4_steps)
    if rank == 0:
        if args.config4_steps > 0:
            out["config4"] = c4
        if not args.no_cpu and world == 1:
            out["cpu_baseline"] = cpu_baseline(N, args.cpu_iters)
        print(json.dumps(out), flush=True)
    dev.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
