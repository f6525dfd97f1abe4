"""Merge the slab digests of N = 1 bench lines into tests/golden/slab_digests.json.

    python scripts/golden_digests.py gpurun_out/.../bench.log [...]

Only lines whose iterate was bitwise equal to the C oracle's are taken
(slab_digests.equal_to_oracle), so every committed digest is of an
oracle-checked iterate; an N-rank bench line compares its rank digests with
them (bench.py, parity "slab sha256 vs N=1")."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLD = os.path.join(ROOT, "tests", "golden", "slab_digests.json")


def main(paths):
    gold = {}
    if os.path.exists(GOLD):
        with open(GOLD) as f:
            gold = json.load(f)
    for p in paths:
        with open(p) as f:
            for ln in f:
                if not ln.startswith("{"):
                    continue
                d = json.loads(ln)
                s = d.get("slab_digests")
                if not s or d.get("n_gpus") != 1 or not s.get("equal_to_oracle"):
                    continue
                old = gold.get(s["key"])
                if old is not None and old != s["digests"]:
                    sys.exit(f"{p}: digests for {s['key']} differ from the committed ones")
                gold[s["key"]] = s["digests"]
                print(f"{s['key']}: {s['digests']['1'][0][:16]}... from {p}")
    with open(GOLD, "w") as f:
        json.dump(gold, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1:])
