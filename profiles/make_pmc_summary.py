"""Summarise rocprofv3 FETCH_SIZE / WRITE_SIZE passes (separate runs) into profiles/pmc_scan.json.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024): on gfx950 FETCH_SIZE tallies the
128-B read requests of wide coalesced loads at 64 B (MI355X_MICROARCH.md §HBM); WRITE_SIZE is
exact for 16-B-per-lane stores.
usage: python profiles/make_pmc_summary.py FETCH_CSV WRITE_CSV SOURCE_NOTE
"""
import collections
import csv
import json
import os
import sys


def per_kernel(path, counter):
    tot, cnt = collections.defaultdict(float), collections.Counter()
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0].replace("void ", "").split("<")[0]
        tot[name] += float(r["Counter_Value"])
        cnt[name] += 1
    return {k: (tot[k] / cnt[k], cnt[k]) for k in tot}


def main():
    fetch, write, note = sys.argv[1], sys.argv[2], sys.argv[3]
    f, w = per_kernel(fetch, "FETCH_SIZE"), per_kernel(write, "WRITE_SIZE")
    out = {"source": note,
           "note": "HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB x 1024), the gfx950 correction of "
                   "MI355X_MICROARCH.md §HBM (128-B read requests tallied at 64 B)",
           "per_kernel": {}}
    for k in sorted(set(f) | set(w)):
        if not k.startswith("ks::"):
            continue
        out["per_kernel"][k] = {"FETCH_SIZE_KB_avg": round(f.get(k, (0, 0))[0], 1),
                                "WRITE_SIZE_KB_avg": round(w.get(k, (0, 0))[0], 1),
                                "launches": f.get(k, (0, 0))[1]}
    s = out["per_kernel"].get("ks::scan_kernel")
    if s:
        out["hbm_bytes_per_scan_launch"] = int((2 * s["FETCH_SIZE_KB_avg"] + s["WRITE_SIZE_KB_avg"]) * 1024)
    dst = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pmc_scan.json")
    with open(dst, "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
