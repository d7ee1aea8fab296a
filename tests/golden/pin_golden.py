"""Check gpurun_out/golden_ref.json (the reference's own kernels and RNG,
tests/golden/make_golden_ref.py, run on MI355X) digest for digest against
tests/golden/golden.json (the CPU oracle, make_golden.py) and record the pin
in golden.json.  Refuses to write on any difference.
usage: python tests/golden/pin_golden.py [gpurun_out/golden_ref.json]"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
ref_path = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "golden_ref.json")
ref = json.load(open(ref_path))
gold_path = os.path.join(HERE, "golden.json")
gold = json.load(open(gold_path))
rows = 0
for name, grows in gold["cases"].items():
    rrows = ref["cases"][name]
    assert len(rrows) == len(grows), name
    for i, (g, r) in enumerate(zip(grows, rrows)):
        assert g == r, (name, i, g, r)
        rows += 1
gold["pinned_by"] = {
    "script": "tests/golden/make_golden_ref.py (GPU) + tests/golden/pin_golden.py",
    "source": ref["source"],
    "rows": rows,
    "result": "every digest identical to the CPU oracle's",
}
with open(gold_path, "w") as f:
    json.dump(gold, f, indent=0, sort_keys=True)
    f.write("\n")
print(f"golden.json pinned: {rows} rows identical")
