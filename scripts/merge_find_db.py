"""Merge kernel-choice find-dbs (bench.py --tune-save output) into the shipped one: entries of the NEW files win
over the base file's entries with the same key; the base's other entries are kept.

    python scripts/merge_find_db.py tuning/mi355x_find_db.json new1.json [new2.json ...]  (rewrites the first)
    python scripts/merge_find_db.py --missing-only BASE new1.json ...  (add only keys the base lacks)
"""
import json
import sys


def main():
    args = sys.argv[1:]
    missing_only = args[0] == "--missing-only"
    if missing_only:
        args = args[1:]
    base_path, news = args[0], args[1:]
    base = json.load(open(base_path))
    for kind in ("conv", "wgrad"):
        merged = {}
        have = {k for k, _ in base.get(kind, [])}
        for path in news:
            for k, v in json.load(open(path)).get(kind, []):
                if not (missing_only and k in have):
                    merged.setdefault(k, v)
        n_new = len(merged)
        kept = 0
        for k, v in base.get(kind, []):
            if k not in merged:
                merged[k] = v
                kept += 1
        base[kind] = [[k, v] for k, v in merged.items()]
        print(f"{kind}: {n_new} new / replaced, {kept} kept from the base", file=sys.stderr)
    with open(base_path, "w") as f:
        json.dump(base, f, indent=0)


if __name__ == "__main__":
    main()
