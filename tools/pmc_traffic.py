"""Reduce rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE runs of bench.py to HBM bytes
per launch (tuning aid; writes profiles/pmc_traffic.json read by bench.py).

    python tools/pmc_traffic.py <FETCH run dir> <WRITE run dir> [out.json]

gfx950 correction (MI355X_MICROARCH.md, HBM/rocprofv3): FETCH_SIZE counts the
fabric read requests at half their bytes -- checked on this code's 8-byte
per-lane copy kernel (k_ew, 80.6 MB read: FETCH_SIZE 40.3 MB) -- so it is
doubled; WRITE_SIZE is exact.  Units: KB.  The ILU apply entry sums the
median per-launch bytes of its four kernels (2 permutations, 2 sweeps).
(The permutations are k_gather4 since round 1's later builds; k_perm before.)"""
import collections
import csv
import glob
import json
import os
import re
import sys


def per_kernel(run_dir):
    f = glob.glob(os.path.join(run_dir, "**", "*counter_collection.csv"), recursive=True)[0]
    agg = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"]].append(float(r["Counter_Value"]) * 1000.0)
    return {k: sorted(v)[len(v) // 2] for k, v in agg.items()}


def main(fetch_dir, write_dir, out):
    fe, wr = per_kernel(fetch_dir), per_kernel(write_dir)

    def find(sub):
        return [k for k in fe if sub in k]

    res = {}
    for k in find("k_spmv3<0, 0"):  # y = A x (any column coding)
        res["k_spmv3"] = int(2 * fe[k] + wr.get(k, 0))
    # line sweeps: the apply's plain rhs gather + one L and one U launch (not
    # BiCGSTAB's p / s passes fused with the gather, k_line_rhs2<RUN, 1 | 2>)
    gathers = [k for k in find("k_line_rhs") if "k_line_rhs<" in k or re.search(r"k_line_rhs2<\d+, 0>", k)]
    line = find("k_line<") + find("k_line2<") + gathers
    if line:
        res["ilu_apply"] = int(sum(2 * fe[k] + wr.get(k, 0) for k in line))
    tri = find("k_tri_pk6")
    perm = find("k_perm")
    g4 = find("k_gather4")  # both permutations of an apply, one kernel: twice its median
    perm_b = 2 * sum(2 * fe[k] + wr.get(k, 0) for k in g4) if g4 else sum(2 * fe[k] + wr.get(k, 0) for k in perm)
    if tri and (perm or g4) and not line:
        res["ilu_apply"] = int(perm_b + 2 * sum(2 * fe[k] + wr.get(k, 0) for k in tri) / max(1, len(tri)))
    res["_note"] = "HBM bytes per launch: 2 x FETCH_SIZE + WRITE_SIZE (rocprofv3 --pmc, medians over launches)"
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json")
