"""Per-launch HBM traffic of a kernel from rocprofv3 --pmc passes.

Usage: python tools/pmc_traffic.py <fetch_csv> <write_csv> <kernel> <out.json> [config batch mode]

``config batch mode`` (default C 65536 single) name the bench.py run the passes profiled;
bench.py only reports a measurement whose keys match its own run
(profiles/traffic/<config>_b<batch>_<mode>_<kernel>.json).

FETCH_SIZE / WRITE_SIZE are in KiB.  gfx950 correction (MI355X_MICROARCH.md
§HBM): FETCH_SIZE reports exactly half the bytes of a wide (16 B/lane)
coalesced streaming read, so it is doubled; WRITE_SIZE is exact for 16-B
stores.  Both kernels this is used for stream their bulk traffic with
16 B/lane accesses.
"""

import csv
import json
import sys


def per_launch(path, counter, kernel):
    vals = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
            if r["Counter_Name"] == counter and kernel in r["Kernel_Name"]]
    if not vals:
        raise SystemExit("no %s rows for %s in %s" % (counter, kernel, path))
    return sum(vals) / len(vals), len(vals)


def main():
    fetch_csv, write_csv, kernel, out = sys.argv[1:5]
    config, batch, mode = (sys.argv[5:8] + ["C", "65536", "single"][len(sys.argv[5:8]):])
    f, nf = per_launch(fetch_csv, "FETCH_SIZE", kernel)
    w, nw = per_launch(write_csv, "WRITE_SIZE", kernel)
    res = {"kernel": kernel, "config": config, "batch": int(batch), "mode": mode, "fetch_size_kib_raw": f, "write_size_kib": w, "launches": [nf, nw],
           "correction": "FETCH_SIZE x2 (gfx950 wide coalesced reads), WRITE_SIZE x1",
           "bytes_per_launch": int((2 * f + w) * 1024)}
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
