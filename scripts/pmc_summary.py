"""Summarise rocprofv3 --pmc runs (FETCH_SIZE and WRITE_SIZE in separate passes) into
profiles/pmc_summary.json: HBM bytes per launch per kernel.

    python scripts/pmc_summary.py <fetch_dir> <write_dir> [out.json] [commit]

The summary carries `_meta`: the digest of the HIP sources it measured (build.sources_digest) and the
commit they were taken from (passed by the round script, since the GPU box has no .git): bench.py
reports `roofline.traffic` only when the running tree's digest equals it.

FETCH_SIZE / WRITE_SIZE are in KiB.  Per MI355X_MICROARCH.md §HBM, gfx950 FETCH_SIZE reports half
the bytes of wide coalesced reads: it is doubled here (an upper bound for narrower access widths,
which are uncalibrated); WRITE_SIZE is taken as is.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def per_kernel(d, counter):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    tot, n = defaultdict(float), defaultdict(int)
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            k = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0]
            k = k.replace("viba::", "").replace("void ", "")
            k = k.split("<")[0].strip()
            tot[k] += float(r["Counter_Value"])
            n[k] += 1
    return {k: (tot[k] / n[k], n[k]) for k in tot}


def main():
    fetch, write = per_kernel(sys.argv[1], "FETCH_SIZE"), per_kernel(sys.argv[2], "WRITE_SIZE")
    out = {}
    for k in sorted(set(fetch) | set(write)):
        fk = fetch.get(k, (0.0, 0))[0] * 1024 * 2
        wk = write.get(k, (0.0, 0))[0] * 1024
        out[k] = {"fetch_bytes_per_launch_x2": fk, "write_bytes_per_launch": wk, "hbm_bytes_per_launch": fk + wk,
                  "launches": max(fetch.get(k, (0, 0))[1], write.get(k, (0, 0))[1])}
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    from visual_inertial_bundle_adjustment_amd.build import sources_digest
    out["_meta"] = {"sources_sha256": sources_digest(), "commit": sys.argv[4] if len(sys.argv) > 4 else None,
                    "counters": "FETCH_SIZE (x2, gfx950) + WRITE_SIZE, separate rocprofv3 --pmc passes of bench.py"}
    path = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_summary.json"
    os.makedirs(os.path.dirname(path), exist_ok=True)
    json.dump(out, open(path, "w"), indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
