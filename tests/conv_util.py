"""Shared helpers of the format-conversion tests (tests/golden/conv.*)."""
import json
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def conv_cases():
    with open(os.path.join(GOLDEN, "conv.json")) as f:
        cases = json.load(f)["cases"]
    with np.load(os.path.join(GOLDEN, "conv.npz"), allow_pickle=False) as z:
        arrays = {k: z[k] for k in z.files}
    for c in cases:
        c["in"] = {k: arrays[f"{c['name']}__{k}"] for k in c["inputs"]}
        c["out"] = {k: arrays[f"{c['name']}__{k}"] for k in c["outputs"]}
    return cases


def same(a, b) -> bool:
    """bitwise equality (NaN payloads included) of int32 / float64 arrays"""
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    if a.dtype == np.float64:
        return np.array_equal(a.view(np.int64), b.view(np.int64))
    return np.array_equal(a, b)
