"""Summarise one profiling run of bench.py (profiles/run_profile.sh) into the
JSON committed under profiles/: per kernel, the average duration from the
kernel trace, the PMC counters summed over the run, and derived figures per
stereo block.

    python profiles/summarize_pmc.py gpurun_out/prof_<TAG> <blocks_total> > profiles/<TAG>_pmc.json

<blocks_total> = stereo blocks encoded by the profiled command over all its
steps (warmup included), e.g. (1 + 2) x 10^6 for "--warmup 1 --steps 2" of
10^6 blocks.  Per-block figures are run totals / blocks_total, so kernels
launched once per chunk (master) and once per step (origin) read alike.

The summary records the source hash of the build that was profiled
(pac_amd.build.source_hash(), printed by bench.py as "src_hash"); bench.py
refuses counters whose hash differs from the running build.

Counter conventions (MI355X_MICROARCH.md, HBM section): FETCH_SIZE and
WRITE_SIZE are in KiB; FETCH_SIZE counts half the bytes of wide coalesced
reads on gfx950, so the read traffic is 2 x FETCH_SIZE.  Calibrated for our
own shapes on a known byte count (tools/probe/fetch_calib.hip,
profiles/r06_fetch_calibration.json): 8 B per lane x2.00, 4 x 16 B per lane
x1.99, 8- and 16-byte-per-lane stores exact; and the doubled figure equals the
algorithmic 4096 B per block within 0.1 % on k_origin_front's PCM loads.
GRBM_GUI_ACTIVE is summed over the 8 XCDs.  FP64 FLOPs = 64 lanes x (ADD +
MUL + 2 FMA) per wave instruction (an upper bound: partially masked waves
count as full).
"""
import collections
import csv
import glob
import json
import os
import re
import subprocess
import sys

SIMDS = 256 * 4


def totals(path):
    """({kernel: {counter: value summed over dispatches}}, {kernel: dispatches})"""
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        k = r["Kernel_Name"].split("(")[0]
        acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    return acc, {k: len(v) for k, v in disp.items()}


def kernel_stats(path):
    out = {}
    for r in csv.DictReader(open(path)):
        out[r["Name"].split("(")[0]] = {"calls": int(r["Calls"]), "avg_ms": float(r["AverageNs"]) / 1e6,
                                        "total_ms": float(r["TotalDurationNs"]) / 1e6,
                                        "pct": float(r["Percentage"])}
    return out


def src_hash_from_log(prefix):
    for f in sorted(glob.glob(prefix + "_*.log")):
        m = re.search(r'"src_hash": "([0-9a-f]+)"', open(f, errors="replace").read())
        if m:
            return m.group(1)
    return None


def derive(c, blocks, total_ms):
    d = {}
    if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
        rd = 2 * c["FETCH_SIZE"] * 1024
        wr = c["WRITE_SIZE"] * 1024
        d["hbm_read_bytes_per_block"] = rd / blocks
        d["hbm_write_bytes_per_block"] = wr / blocks
    if "SQ_INSTS_VALU_FMA_F64" in c:
        fl = 64 * (c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + 2 * c["SQ_INSTS_VALU_FMA_F64"])
        d["fp64_flop_per_block"] = fl / blocks
        if total_ms:
            d["fp64_tflops"] = fl / (total_ms / 1e3) / 1e12
    if "SQ_INSTS_VALU" in c:
        d["valu_insts_per_block"] = c["SQ_INSTS_VALU"] / blocks
        if "SQ_INSTS_VALU_ADD_F64" in c:
            f64 = c["SQ_INSTS_VALU_ADD_F64"] + c["SQ_INSTS_VALU_MUL_F64"] + c["SQ_INSTS_VALU_FMA_F64"] + \
                c.get("SQ_INSTS_VALU_TRANS_F64", 0.0)
            d["fp64_share_of_valu"] = f64 / c["SQ_INSTS_VALU"]
    if "SQ_INSTS_VALU" in c and "GRBM_GUI_ACTIVE" in c and total_ms:
        cyc = c["GRBM_GUI_ACTIVE"] / 8
        d["clock_ghz"] = cyc / (total_ms / 1e3) / 1e9
        d["valu_issue_util"] = c["SQ_INSTS_VALU"] * 4 / (SIMDS * cyc)
    if "SQ_LDS_BANK_CONFLICT" in c and c.get("SQ_LDS_IDX_ACTIVE"):
        # extra cycles / all LDS-array cycles (MI355X_MICROARCH.md LDS section)
        d["lds_bank_conflict_frac"] = c["SQ_LDS_BANK_CONFLICT"] / c["SQ_LDS_IDX_ACTIVE"]
    if "SQ_WAVE_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
        # achieved occupancy: resident waves per SIMD averaged over the kernel's
        # busy time (SQ_WAVE_CYCLES counts quad-cycles, MI355X_MICROARCH.md;
        # under --pmc the dispatches run one at a time, so GRBM_GUI_ACTIVE / 8
        # is this kernel's own duration in cycles)
        d["waves_per_simd"] = 4 * c["SQ_WAVE_CYCLES"] / (SIMDS * c["GRBM_GUI_ACTIVE"] / 8)
    if "SQ_WAIT_ANY" in c and c.get("SQ_WAVE_CYCLES"):
        d["wait_frac"] = c["SQ_WAIT_ANY"] / c["SQ_WAVE_CYCLES"]
    return d


def main(prefix, blocks):
    blocks = float(blocks)
    res = {"source": prefix, "blocks_total": blocks, "kernels": {}}
    try:
        res["commit"] = subprocess.run(["git", "rev-parse", "--short", "HEAD"], capture_output=True,
                                       text=True).stdout.strip()
    except OSError:
        pass
    res["src_hash"] = src_hash_from_log(prefix)
    ks = glob.glob(prefix + "_kt/*kernel_stats.csv")
    stats = kernel_stats(ks[0]) if ks else {}
    counters = collections.defaultdict(dict)
    for f in sorted(glob.glob(prefix + "_*/*counter_collection.csv")):
        acc, _ = totals(f)
        for k, d in acc.items():
            counters[k].update(d)
    for k in sorted(set(stats) | set(counters)):
        st = stats.get(k)
        c = counters.get(k) or {}
        res["kernels"][k] = {"trace": st, "pmc_total": c,
                             "derived": derive(c, blocks, st["total_ms"] if st else None)}
    json.dump(res, sys.stdout, indent=1, sort_keys=True)
    print()


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
