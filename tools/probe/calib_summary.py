"""Summarise the FETCH_SIZE / WRITE_SIZE calibration run (tools/calib.sh,
tools/probe/fetch_calib.hip) into the factors bytes / counter-bytes per access
shape:

    python tools/probe/calib_summary.py gpurun_out > profiles/r06_fetch_calibration.json

Counters are in KiB; every probe kernel touches exactly 2^30 bytes.
"""
import collections
import csv
import glob
import json
import sys

NBYTES = 1 << 30
SHAPES = {"k_rd8": "read, 64 lanes x 8 B contiguous per wave instruction (k_master_thr's threshold-row reads)",
          "k_rd16": "read, 64 lanes x 16 B contiguous (MI355X_MICROARCH.md's calibrated shape)",
          "k_rd16x4": "read, 4 consecutive 16 B per lane, lanes 64 B apart (k_master_thr's spectra reads)",
          "k_wr8": "write, 64 lanes x 8 B contiguous (k_master_thr's threshold-row writes)",
          "k_wr16": "write, 64 lanes x 16 B contiguous"}


def counters(d):
    acc = collections.defaultdict(float)
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[(r["Kernel_Name"].split("(")[0], r["Counter_Name"])] += float(r["Counter_Value"])
    return acc


def main(out):
    fetch, write = counters(out + "/calib_fetch"), counters(out + "/calib_write")
    res = {"bytes_per_kernel": NBYTES, "source": "tools/calib.sh (tools/probe/fetch_calib.hip), one rocprofv3 "
           "--pmc pass per counter", "kernels": {}}
    for k, shape in SHAPES.items():
        f = fetch.get((k, "FETCH_SIZE"))
        w = write.get((k, "WRITE_SIZE"))
        e = {"shape": shape, "FETCH_SIZE_bytes": f * 1024 if f is not None else None,
             "WRITE_SIZE_bytes": w * 1024 if w is not None else None}
        if k.startswith("k_rd") and f:
            e["bytes_per_FETCH_SIZE_byte"] = NBYTES / (f * 1024)
        if k.startswith("k_wr") and w:
            e["bytes_per_WRITE_SIZE_byte"] = NBYTES / (w * 1024)
        res["kernels"][k] = e
    json.dump(res, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1])
