"""Regenerate tests/golden/golden.json.

For every reference test case in cases.CASES and every one of its 128
iterations, record n (and startBit) plus sha256[:16] of the sorted keys and
values.  Each expected output is computed by the oracle's LSD restatement AND
checked, at generation time, against the reference tests' own CPU oracles
(std::sort / std::stable_sort / stableSortPairs, unittest.cpp:154-161,
283-291, 343-348, 358-377) and the numpy contract; the script refuses to write
a fixture those disagree on.

Also records the SURVEY.md s4 anchors (splitmix64 outputs, SortKeys.u32
iteration 0/1), which were computed independently by a Python restatement in
the survey session.

Usage: python tests/golden/make_golden.py   (about a minute on 8 cores)
"""
from __future__ import annotations

import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import cases as C  # noqa: E402
from cases import O  # noqa: E402


def check_against_reference_oracles(name: str, item: dict, k_out: np.ndarray, v_out):
    kind, kt, vb, desc, _ = C.CASES[name]
    keys = item["keys"]
    if kind == "keys":
        ref = O.std_sort_keys(kt, keys, desc)
        if kt in (O.F32, O.F64):   # compare as floats: == treats -0 and +0 alike (unittest.cpp:165)
            ft = np.float32 if kt == O.F32 else np.float64
            assert np.array_equal(ref.view(ft), k_out.view(ft)), name
        else:
            assert np.array_equal(ref, k_out), name
    elif kind == "window":
        ref_k, ref_v = O.std_stable_sort_window_u64(keys, item.get("values"), int(item["start"]), desc)
        assert np.array_equal(ref_k, k_out), name
        if v_out is not None:
            assert np.array_equal(ref_v, v_out), name
    else:
        ref_k, ref_v = O.std_stable_sort_pairs(kt, keys, item["values"])
        assert np.array_equal(ref_k, k_out), name
        assert np.array_equal(ref_v, v_out), name
    # numpy contract (stable argsort by digits of the transformed key)
    if kind == "window":
        s = int(item["start"])
        order = O.contract_sort_order(kt, keys, s, s + 8, desc)
    else:
        order = O.contract_sort_order(kt, keys, 0, O.KEY_BYTES[kt] * 8, desc)
    assert np.array_equal(keys[order], k_out), name


def main():
    out = {"generator": "tests/golden/make_golden.py", "oracle": "oracle/oracle.cpp orc_lsd_sort",
           "cases": {}}
    r = O.SplitMix64()
    out["anchors"] = {
        "splitmix64_first3": [hex(r.next()) for _ in range(3)],
    }
    for name, (kind, kt, vb, desc, stream) in C.CASES.items():
        rows = []
        for item in stream():
            k_out, v_out = C.oracle_result(name, item)
            check_against_reference_oracles(name, item, k_out, v_out)
            row = {"n": int(item["n"]), "keys": C.digest(k_out)}
            if "start" in item:
                row["start"] = int(item["start"])
            if v_out is not None:
                row["values"] = C.digest(v_out)
            rows.append(row)
        out["cases"][name] = rows
        print(f"{name}: {len(rows)} iterations", flush=True)
    first = out["cases"]["SortKeys.u32"]
    out["anchors"]["SortKeys.u32.iter0"] = {"n": first[0]["n"], "sha256_16": first[0]["keys"]}
    out["anchors"]["SortKeys.u32.iter1"] = {"n": first[1]["n"], "sha256_16": first[1]["keys"]}
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=0, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main()
