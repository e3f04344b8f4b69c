"""Merge the result rows of TunableOp CSVs (tools/tune_gemms.py outputs) into the packaged table
(shuffle_exchange_amd/tuning/tunableop_mi355x.csv): the packaged Validator lines are kept, a row
with the same (op, shape) key is replaced by the newer one.
  python tools/merge_tunableop.py NEW.csv [NEW2.csv ...]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TABLE = os.path.join(ROOT, "shuffle_exchange_amd", "tuning", "tunableop_mi355x.csv")


def rows(path):
    head, body = [], {}
    for line in open(path):
        line = line.rstrip("\n")
        if not line:
            continue
        f = line.split(",")
        if f[0] == "Validator":
            head.append(line)
        elif len(f) >= 3:
            body[(f[0], f[1])] = line
    return head, body


def main():
    head, body = rows(TABLE)
    for p in sys.argv[1:]:
        h, b = rows(p)
        new_val = {l.split(",")[1]: l for l in h}
        for l in head:  # the tuned solutions are only valid for the same library versions
            k = l.split(",")[1]
            if k in new_val and new_val[k] != l and k != "PT_VERSION":
                raise SystemExit(f"{p}: validator {k} differs from the packaged table ({new_val[k]} vs {l})")
        added = sum(1 for k in b if k not in body)
        body.update(b)
        print(f"{p}: {len(b)} rows ({added} new)")
    with open(TABLE, "w") as f:
        f.write("\n".join(head + sorted(body.values())) + "\n")
    print(f"{TABLE}: {len(body)} tuned shapes")


if __name__ == "__main__":
    main()
