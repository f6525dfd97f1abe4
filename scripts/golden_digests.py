"""Merge the slab digests of one-GPU bench lines into tests/golden/slab_digests.json.

    python scripts/golden_digests.py gpurun_out/.../bench.log [...]

Column "1" comes from the one-process bench line, column "N" from a
`bench.py --emulate N` line (the N-rank setup under the rank emulation, whose
iterate an N-rank run must reproduce bit for bit).  Only lines whose iterate
was bitwise equal to the C oracle's are taken (slab_digests.equal_to_oracle),
so every committed digest is of an oracle-checked iterate; an N-rank bench
line compares its rank digests with column N (bench.py parity)."""
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
                ent = gold.setdefault(s["key"], {})
                for col, dig in s["digests"].items():
                    if col in ent and ent[col] != dig:
                        sys.exit(f"{p}: column {col} of {s['key']} differs from the committed one")
                    ent[col] = dig
                    print(f"{s['key']} [{col}]: {dig[0][:16]}... from {p}")
    with open(GOLD, "w") as f:
        json.dump(gold, f, indent=1, sort_keys=True)
        f.write("\n")


if __name__ == "__main__":
    main(sys.argv[1:])
