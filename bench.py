#!/usr/bin/env python3
"""Benchmark: stereo 1024-sample blocks encoded per second on MI355X.

Workloads (BASELINE.json configs; --config picks one, default 2):

  2  (default, the largest single-GPU config -- BASELINE.json's metric names
     no config): synthetic 48 kHz stereo pink noise + 440/1250/5300 Hz tones,
     10^7 stereo blocks per GPU as 10 000 independent streams x 1000 blocks
     (999 hops + the Close() flush block each), master profile: full
     psychoacoustics (6 masking thresholds), M/S decision, reservoir bit
     allocation, Huffman (.wak) -- the reference's codec/ coder.
  1  synthetic 48 kHz stereo white noise, 10^6 blocks per GPU (1000 x 1000),
     origin profile ("M/S off": PerceptualAudioCodec_Origin's coder).
  3  the reference's inputs/*.wav (stereo ones, shipped under
     tests/fixtures/inputs/) x --copies, each copy an independent master +
     Huffman stream (per-file reservoir exactly as the reference), whole
     streams sharded over the ranks by pac_amd.shard.plan (LPT).
  4  block switching (an extension, parity unpinned -- pac_bs.h): synthetic
     48 kHz stereo pink noise + tones + one decaying noise burst per 8192
     frames, N=1024/256 block switching with attack detection, master
     profile; 1.25 x 10^7 stereo blocks per GPU (12 500 streams x 1000
     blocks), i.e. 10^8 over the 8 GPUs of configs[4].

The PCM is generated on (configs 1-2) or uploaded to (config 3) the device
before the timed region, so the timed region starts with the inputs resident
in HBM; one step = the pac_encode_streams call(s) over all of this rank's
blocks (MDCT, masking thresholds, bit allocation, quantization, Huffman, bit
packing into the .pac/.wak data sections, all in HBM).

    python bench.py [--config C] [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Streams shard across ranks with no data-path collective (weak scaling for
configs 1-2, strong for config 3); the only cross-rank traffic is the barrier
and the max-over-ranks of the timer (gloo, CPU tensors).  Rank 0 prints one
JSON line.
"""
import argparse
import ctypes as C
import glob
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import pac_amd  # noqa: E402,F401
from pac_amd import _lib, build as _build, shard  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector peak (spec)
INPUTS = os.path.join(ROOT, "tests", "fixtures", "inputs")


def host_cores():
    """CPUs this process may use: the affinity set, capped by the host's
    OMP_NUM_THREADS share when set (the GPU box exports 16 and shows the whole
    machine's CPUs in the affinity set)"""
    n = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    return min(n, int(omp)) if omp.isdigit() and int(omp) > 0 else n


def cgroup_cpus():
    """The CPU quota of this process's cgroup (cgroup v2 cpu.max, v1
    cfs_quota/period) in CPUs, or None when unlimited / unreadable"""
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        return None if q == "max" else int(q) / int(per)
    except (OSError, ValueError):
        pass
    try:
        with open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us") as f:
            q = int(f.read())
        with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
            per = int(f.read())
        return None if q <= 0 else q / per
    except (OSError, ValueError):
        return None


def cpu_share():
    """What the CPU baseline's thread count is measured against: nproc, the
    affinity set, OMP_NUM_THREADS and the cgroup quota, and why the baseline
    runs on host_cores() threads"""
    omp = os.environ.get("OMP_NUM_THREADS")
    quota = cgroup_cpus()
    aff = len(os.sched_getaffinity(0))
    why = []
    if omp and omp.isdigit() and int(omp) < aff:
        why.append("OMP_NUM_THREADS=%s is this host's per-job CPU share (the GPU box exports it; its affinity "
                   "set shows the whole machine's %d CPUs, shared with the other GPUs' jobs)" % (omp, aff))
    if quota is not None:
        why.append("cgroup CPU quota %.1f CPUs" % quota)
    if not why:
        why.append("every CPU of the affinity set")
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "omp_num_threads": omp,
            "cgroup_quota_cpus": quota, "threads_used": host_cores(), "why": "; ".join(why)}


# the reference Python itself, timed in the survey container:
# it cannot run on the GPU box (Python 2 source, /root/reference absent there)
REF_PYTHON = {"master": {"value": 11.0, "unit": "blocks/s", "cores": 1,
                         "sample": "BASELINE.md: reference codec/ (Py3 semantics shim) on inputs/harpsichord.wav, "
                                   "387 blocks, 1 core of the survey container's Xeon"},
              "origin": {"value": 18.1, "unit": "blocks/s", "cores": 1,
                         "sample": "BASELINE.md: reference PerceptualAudioCodec_Origin/codec/ on "
                                   "inputs/harpsichord.wav, 387 blocks, 1 core of the survey container's Xeon"}}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", type=int, choices=[1, 2, 3, 4], default=2,
                    help="BASELINE.json configs[i]: 1 origin white noise 10^6, 2 master pink+tones 10^7 "
                         "(default), 3 master real-audio file batch, 4 block switching 1.25x10^7 per GPU")
    ap.add_argument("--mode", choices=["encode", "decode"], default="encode",
                    help="encode = the metric (default); decode = pac_decode_streams of the same "
                         "workload's bitstream (encoded once, untimed)")
    ap.add_argument("--profile", choices=["origin", "master"], default=None,
                    help="legacy alias: origin = --config 1, master = --config 2")
    ap.add_argument("--streams", type=int, default=None,
                    help="configs 1/2: streams per GPU (default 1000 / 10000)")
    ap.add_argument("--blocks-per-stream", type=int, default=1000)
    ap.add_argument("--copies", type=int, default=1000, help="config 3: copies of every input file")
    ap.add_argument("--sample-rate", type=int, default=48000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="decode mode: bounded CPU-baseline sample (oracle on host cores)")
    ap.add_argument("--cpu-blocks", type=int, default=-1,
                    help="encode CPU baseline: blocks per sampled stream (default -1: whole streams, "
                         "~10-15 s on 16 host threads for configs[2])")
    ap.add_argument("--parity-streams", type=int, default=64,
                    help="whole streams re-encoded by the CPU oracle and compared with the GPU's bytes, over "
                         "all ranks (each rank samples ceil(n / world), at least 16, of its own streams)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="host threads of the CPU baseline (default: the CPUs this process may run on, "
                         "os.sched_getaffinity, capped by OMP_NUM_THREADS when the host sets it -- the "
                         "GPU box's CPU share)")
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    if a.profile is not None:
        a.config = 1 if a.profile == "origin" else 2
    if a.cpu_threads is None:
        a.cpu_threads = host_cores()
    a.master = a.config != 1
    a.bs = a.config == 4
    a.profile = "master" if a.master else "origin"
    if a.streams is None:
        a.streams = {2: 10000, 4: 12500}.get(a.config, 1000)
    return a


def free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(a):
    """`bench.py --gpus N` (N > 1) outside torchrun: start N fresh rank
    processes of this same script (RANK = LOCAL_RANK = r, WORLD_SIZE = N,
    MASTER_ADDR 127.0.0.1, device = LOCAL_RANK), relay rank 0's stdout (the one
    JSON line) and return the first non-zero exit status.  This parent never
    initialises the GPU (the library loads lazily, in the ranks), so starting
    children is safe; if one rank fails the others are terminated -- they would
    otherwise wait at the barrier."""
    import signal
    import subprocess
    import threading
    port = os.environ.get("MASTER_PORT") or str(free_port())
    argv = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    procs, out0 = [], []

    def stop(*_):
        raise SystemExit(143)

    prev = signal.signal(signal.SIGTERM, stop)
    try:
        for r in range(a.gpus):
            env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(a.gpus),
                       LOCAL_WORLD_SIZE=str(a.gpus), GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
            procs.append(subprocess.Popen(argv, env=env, stdout=subprocess.PIPE if r == 0 else sys.stderr,
                                          text=True))
        rd = threading.Thread(target=lambda: out0.extend(procs[0].stdout), daemon=True)
        rd.start()
        rc = 0
        while any(p.poll() is None for p in procs):
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0]
                print("bench.py: a rank exited with %d; stopping the others" % rc, file=sys.stderr, flush=True)
                break
            time.sleep(0.2)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
        signal.signal(signal.SIGTERM, prev)
    rd.join(timeout=10)
    sys.stdout.write("".join(out0))
    sys.stdout.flush()
    return rc or next((p.returncode for p in procs if p.returncode), 0)


def make_context(dev, huffman):
    """The device context of this rank.  PAC_BENCH_MOCK_CONTEXT=<file.py> is a
    TEST-ONLY hook (tests/bench_mock.py): it replaces the HIP context by the
    file's Context class so that the rank plumbing (spawn, gloo, parity
    merge) runs on a CPU-only container; a line made that way says so in
    "mock_context" and is never a measurement."""
    mock = os.environ.get("PAC_BENCH_MOCK_CONTEXT")
    if not mock:
        return _lib.Context(dev, huffman=huffman)
    import importlib.util
    spec = importlib.util.spec_from_file_location("pac_bench_mock", mock)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m.Context(dev, huffman=huffman)


class Dist:
    """Barrier + max over ranks; gloo on CPU when launched under torchrun (or
    by spawn_ranks)."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.td = None
        if self.world > 1:
            import torch.distributed as td
            # gloo's connection banner goes to fd 1: keep stdout for the one JSON line
            sys.stdout.flush()
            saved = os.dup(1)
            os.dup2(2, 1)
            try:
                td.init_process_group("gloo")
            finally:
                sys.stdout.flush()
                os.dup2(saved, 1)
                os.close(saved)
            self.td = td

    def barrier(self):
        if self.td:
            self.td.barrier()

    def _red(self, v, op):
        if not self.td:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.td.all_reduce(t, op=op)
        return float(t.item())

    def max(self, v):
        return self._red(v, self.td.ReduceOp.MAX if self.td else None)

    def sum(self, v):
        return self._red(v, self.td.ReduceOp.SUM if self.td else None)

    def gather(self, obj):
        """every rank's obj, in rank order (gloo all_gather_object)"""
        if not self.td:
            return [obj]
        out = [None] * self.world
        self.td.all_gather_object(out, obj)
        return out

    def close(self):
        if self.td:
            self.td.destroy_process_group()


# the reference's direct masking sum costs ~35 FP64
# flops per (masker, line) pair: origin ~2 x 255 x 1024 pairs per stereo block
# (~18 MFLOP), master 6 x ~222 x 1024 (~48 MFLOP).  Our kernels evaluate the
# same sums in factored forms; "ref_alg_equiv_tflops" prices our
# rate at the reference algorithm's flop count.
REF_ALG_FLOP_PER_BLOCK = {"origin": 18.0e6, "master": 48.0e6}

# Algorithmic HBM bytes per stereo block: the
# 4096 B of int16 PCM read + the packed bitstream written (the measured
# out_bytes / blocks, ~592 B for configs[2]) -- the whole path's bytes, and
# the numerator of roofline.achieved for the dominant kernel too.
PCM_BYTES_PER_BLOCK = 2 * 1024 * 2

# What each kernel of OUR kernel split reads and writes per stereo block
# (inputs + outputs, incl. the intermediates another kernel produced or
# consumes: spectra, threshold rows, MDCT lines).  Not algorithmic bytes --
# reported as roofline.kernel_io_bytes_per_block beside them.
KERNEL_IO_BYTES = {
    "k_origin_front": 4096 + 2 * (25 * 8 * 2 + 1),   # int16 PCM in; SMR + band peaks + overall out
    "k_master_spec": 4096 + 2 * 1025 * 16,           # int16 PCM in; FFT bins 0..1024 of a and b out
    "k_master_thr": 2 * 1025 * 16 + 6 * 1024 * 8,    # the spectra in; 6 threshold rows out (calcBTHR x 6)
    "k_master_front": 4096 + 6 * 1024 * 8 + 2 * 1024 * 8 + 4 * 25 * 8 + 25 + 2,
    "k_master_tail": 2 * 1024 * 8 + 4 * 25 * 8 + 25 + 2 * (25 * 2 + 1 + 4 + 8),
    "k_master_emit": 2 * 1024 * 2 + 2 * (25 * 2 + 1 + 4 + 8) + 25 + 2 * 300,   # codes + fields in; staged bytes out
    "k_master_place": 2 * 2 * (300 + 8 + 4),                                     # staged bytes in, file bytes out
}


def chunk_blocks_of(bs):
    """run_master's chunk size: PAC_CHUNK_BLOCKS, else 32768 (65536 with block
    switching) -- pac_abi.hip run_master"""
    env = os.environ.get("PAC_CHUNK_BLOCKS", "")
    if env.isdigit() and int(env) > 0:
        return int(env)
    return 65536 if bs else 32768


def master_launches(nb, chunk_blocks=32768):
    """launches of each pass-1 master kernel per pac_encode_streams call of
    streams with nb[i] blocks: one per chunk (run_master in pac_abi.hip:
    groups of <= chunk_blocks streams ordered by length, longest first; chunk
    = S blocks of every stream still running at t0, S = min(chunk_blocks /
    running streams, blocks left of the longest))"""
    n = 0
    for g0 in range(0, len(nb), chunk_blocks):
        grp = sorted(nb[g0:g0 + chunk_blocks], reverse=True)
        gmax = max(1, grp[0])
        n_act, t0 = len(grp), 0
        while t0 < gmax:
            while n_act > 1 and grp[n_act - 1] <= t0:
                n_act -= 1
            t0 += max(1, min(chunk_blocks // n_act, gmax - t0))
            n += 1
    return n


def measured_profile(kind, kernel):
    """Per-block HBM bytes and FP64 work of `kernel` from the newest committed
    rocprofv3 PMC summary profiles/r*_<kind>_pmc.json (profiles/run_profile.sh
    + profiles/summarize_pmc.py), used only if its recorded source hash equals
    this build's: counters from another build are reported as stale, never
    combined with this build's times."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_%s_pmc.json" % kind)))
    if not files:
        return None, "no profiles/r*_%s_pmc.json" % kind
    with open(files[-1]) as f:
        d = json.load(f)
    rel = os.path.relpath(files[-1], ROOT)
    if d.get("src_hash") != _build.source_hash():
        return None, "%s is stale (src_hash %s, this build %s)" % (rel, d.get("src_hash"), _build.source_hash())
    ks = d.get("kernels", {})
    k = ks.get(kernel) or ks.get("void " + kernel)   # templates: "void k<..>"
    if not k:                                        # a template named without its arguments: the one instantiation profiled
        inst = [v for n, v in ks.items() if n.startswith("void " + kernel + "<")]
        k = inst[0] if len(inst) == 1 else None
    if not k or not k.get("derived"):
        return None, "%s has no counters for %s" % (rel, kernel)
    out = dict(k["derived"])
    c = k.get("pmc_total") or {}
    if "waves_per_simd" not in out and c.get("SQ_WAVE_CYCLES") and c.get("GRBM_GUI_ACTIVE"):
        out["waves_per_simd"] = 4 * c["SQ_WAVE_CYCLES"] / (1024 * c["GRBM_GUI_ACTIVE"] / 8)   # summarize_pmc.py
    out["_file"] = rel
    return out, rel


def binding(dom, prof):
    """What binds the dominant kernel, only as far as its same-hash PMC
    profile shows it: VALU issue near saturation -> the VALU pipe (FP64 work
    for the threshold kernels); otherwise unknown (null)."""
    if not prof or prof.get("valu_issue_util") is None:
        return None
    u = prof["valu_issue_util"]
    if u < 0.6:
        return {"resource": None, "valu_issue_util": u,
                "note": "%s issues VALU %.0f %% of its cycles: latency/occupancy bound, not VALU" % (dom, 100 * u)}
    return {"resource": "fp64-valu" if prof.get("fp64_share_of_valu", 0) > 0.3 else "valu",
            "valu_issue_util": u, "fp64_share_of_valu": prof.get("fp64_share_of_valu"),
            "note": "%s issues VALU %.0f %% of its cycles (same-hash PMC): bound by VALU issue, not by HBM -- "
                    "the HBM fraction is small by construction (SURVEY.md 8(d), DESIGN.md section 4)"
                    % (dom, 100 * u)}


def csrc_defines(names, files=("pac_wave.h", "pac_common.h", "pac_master.hip")):
    """integer values of the object-like #defines `names` of the kernel
    sources, evaluated through the other #defines they use (so the numbers
    bench.py reports follow the kernels' own constants)"""
    import re
    defs = {}
    for fn in files:
        with open(os.path.join(os.path.dirname(_build.SRC), fn)) as f:
            for line in f:
                m = re.match(r"\s*#define\s+(\w+)\s+([^/\n]+)", line)
                if m and re.fullmatch(r"[\w\s()+\-*/%]+", m.group(2).strip()):
                    defs.setdefault(m.group(1), m.group(2).strip())

    def ev(name, depth=0):
        expr = re.sub(r"[A-Za-z_]\w*", lambda t: "(%d)" % ev(t.group(0), depth + 1), defs[name])
        return int(eval(expr.replace("/", "//"), {"__builtins__": {}}))
    return {n: ev(n) for n in names}


# kernels launched with dynamic LDS (bytes per workgroup, waves per workgroup):
# the compiler's resource report shows 0 for them.  k_master_tail: PAC_TAIL_LDS
# (csrc/pac_master.hip, 22 500 B: smr, group maxima, bits, group indices,
# nLines, the line quarters' Huffman sums) and PAC_TAIL_Q waves per workgroup
# (pac_abi.hip run_master launch), read from the source
def dynamic_lds():
    d = csrc_defines(["PAC_TAIL_LDS", "PAC_TAIL_Q"])
    return {"k_master_tail": (d["PAC_TAIL_LDS"], d["PAC_TAIL_Q"])}

# kernels whose occupancy the line reports beside the dominant one
OCC_KERNELS = ["k_master_lrms_spec", "k_master_front", "k_master_tail", "k_origin_front", "k_master_thr_short"]


def kernel_resources():
    """the compiler's per-kernel VGPRs / LDS / occupancy limit of this build
    (build.py writes it beside the library), {} when missing or stale"""
    try:
        with open(_build.RESOURCES) as f:
            d = json.load(f)
    except (OSError, ValueError):
        return {}
    return d.get("kernels", {}) if d.get("src_hash") == _build.source_hash() else {}


def occupancy(kind, kernels):
    """Per-GPU occupancy (SURVEY 8(d) "Reported", BASELINE configs[4]): the
    achieved resident waves per SIMD of each kernel from the same-hash PMC
    profile (4 x SQ_WAVE_CYCLES / (SIMDs x the kernel's own cycles)), beside
    the limit its resources allow (compiler report: VGPRs; LDS per CU)"""
    res = kernel_resources()
    out = {"unit": "resident waves per SIMD (of 8 slots), averaged over the kernel's own busy time",
           "source": None, "kernels": {}}
    for k in kernels:
        name = k
        r = res.get(k) or next((v for n, v in res.items() if n.startswith(k + "<true>")), None) or \
            next((v for n, v in res.items() if n.startswith(k + "<")), {})
        m, src = measured_profile(kind, k)
        if m is None:
            m, src2 = measured_profile(kind, k + "<true>")
            if m is not None:
                src, name = src2, k + "<true>"
        e = {"achieved_waves_per_simd": m.get("waves_per_simd") if m else None,
             "valu_issue_util": m.get("valu_issue_util") if m else None,
             "limit_waves_per_simd": r.get("occupancy_waves_per_simd"), "vgprs": r.get("vgprs"),
             "lds_bytes_per_workgroup": r.get("lds_bytes")}
        lds = r.get("lds_bytes") or 0
        dyn = dynamic_lds()
        if k in dyn:                  # launched with dynamic LDS: the compiler reports 0
            lds, wg_waves = dyn[k]
            e["lds_bytes_per_workgroup"] = lds
            e["lds_dynamic"] = True
            lim = (160 * 1024) // lds * wg_waves / 4.0       # workgroups per CU x waves each / 4 SIMDs
            e["lds_limit_waves_per_simd"] = lim
            if e["limit_waves_per_simd"] is not None:
                e["limit_waves_per_simd"] = min(e["limit_waves_per_simd"], lim)
        elif lds and k not in ("k_master_tail", "k_master_emit"):     # 256-thread workgroups: 4 waves, one per SIMD
            e["lds_limit_waves_per_simd"] = min(8, (160 * 1024) // lds)
        if m is not None:
            out["source"] = src
        out["kernels"][name] = e
    return out


def cpu_baseline(ctx, samples, fs, profile, threads, bs=False, max_blocks=-1):
    """The CPU oracle (oracle/pac_oracle.c) on a bounded sample of the same
    workload, one host thread per sampled stream (ctypes releases the GIL; the
    C oracle keeps no global state): thread t encodes its whole stream (int16
    frames copied back from HBM; at most max_blocks blocks when >= 0).
    Returns the baseline and each thread's data section (the parity sample)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as P
    from concurrent.futures import ThreadPoolExecutor
    P.lib()
    threads = max(1, min(threads, len(samples)))
    prof = P.MASTER if profile == "master" else P.ORIGIN
    t0 = time.perf_counter()

    def work(t):
        o = P.Oracle(fs, huffman=(prof == P.MASTER), block_switch=bs)
        pcm = samples[t]
        full = (pcm.shape[0] + 1023) // 1024 + 1
        n = full if max_blocks < 0 else min(full, max_blocks)
        return n, o.encode_data(prof, pcm, max_blocks=n)

    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(work, range(len(samples))))
    el = time.perf_counter() - t0
    done = sum(r[0] for r in res)
    base = {"value": done / el, "unit": "blocks/s", "cores": threads, "kind": "port",
            "host_cpus_visible": len(os.sched_getaffinity(0)),
            "reference_python": REF_PYTHON[profile],
            "sample": "oracle/pac_oracle.c (C restatement, byte-exact on the 16 reference "
                      "fixtures), %s profile%s, %d host threads, one sampled stream each (whole streams%s), "
                      "%d stereo blocks in %.1f s"
                      % (profile, " + block switching" if bs else "", threads,
                         "" if max_blocks < 0 else ", <= %d blocks" % max_blocks, done, el)}
    return base, [r[1] for r in res]


def sample_streams(ns, n):
    """n stream indices spread over a batch of ns: the first and the last, the
    one-lane reservoir tail's wave boundaries (lanes 63/64 and 4095/4096 --
    equal-length streams keep their index order in run_master's length sort),
    then an even stride"""
    pick = [i for i in dict.fromkeys([0, ns - 1, 63, 64, 4095, 4096]) if 0 <= i < ns][:n]
    for k in range(n, 4 * n + 2):          # the stride, denser until n distinct indices
        if len(pick) >= min(n, ns):
            break
        for x in np.linspace(0, ns - 1, k - len(pick) + 2)[1:-1]:
            if int(round(x)) not in pick and len(pick) < n:
                pick.append(int(round(x)))
    return sorted(pick)


def channel_blocks(b):
    """split a data section into its '<L nBytes' + payload channel-blocks"""
    out, pos = [], 0
    while pos + 4 <= len(b):
        n = int.from_bytes(b[pos:pos + 4], "little")
        out.append(b[pos:pos + 4 + n])
        pos += 4 + n
    return out


def parity_check(ctx, out_dev, starts, oracle_sections, streams):
    """The oracle's bytes for the sampled streams against the GPU's bytes for
    the same streams: channel-blocks compared and how many differ (SURVEY 8(d):
    flip rate)."""
    checked = bad = 0
    bad_streams = []
    for st, ref, sid in zip(starts, oracle_sections, streams):
        if not ref:
            continue
        got = np.empty(len(ref), dtype=np.uint8)
        ctx.to_host(got, out_dev + int(st))
        a, b = channel_blocks(ref), channel_blocks(got.tobytes())
        checked += len(a)
        nb = sum(1 for x, y in zip(a, b) if x != y) + max(0, len(a) - len(b))
        bad += nb
        if nb:
            bad_streams.append(sid)
    return {"checked_channel_blocks": checked, "mismatching": bad, "streams": streams,
            "mismatching_streams": bad_streams}


def rank_parity(a, ctx, j, rank, world, threads, dist=None):
    """This rank's parity sample: whole streams of its own shard (job j),
    re-encoded by the CPU oracle on `threads` host threads and compared with
    the GPU's bytes.  The first `threads` streams (one per thread) are timed as
    the CPU baseline; with `dist`, rank 0 times its baseline while the other
    ranks wait at a barrier, so its host threads do not share the CPUs with
    their re-encodes.  Returns (baseline, parity dict)."""
    n = min(j.ns, max(16, -(-a.parity_streams // world)))
    idx = sample_streams(j.ns, n)
    nt = max(1, min(threads, len(idx)))

    def timed():
        return cpu_baseline(ctx, j.cpu_samples(idx[:nt]), j.p.sample_rate, a.profile, nt, bs=a.bs,
                            max_blocks=a.cpu_blocks)
    if rank == 0:
        base, sec0 = timed()
    if dist is not None:
        dist.barrier()
    if rank != 0:
        base, sec0 = timed()
    sections = list(sec0)
    rest = idx[nt:]          # the rest of the parity sample, untimed, 4 streams per thread at a time
    for g0 in range(0, len(rest), 4 * nt):
        _, more = cpu_baseline(ctx, j.cpu_samples(rest[g0:g0 + 4 * nt]), j.p.sample_rate, a.profile, nt, bs=a.bs,
                               max_blocks=a.cpu_blocks)
        sections += more
        # progress (a large --parity-streams sample runs for minutes)
        print("rank %d parity: %d / %d streams re-encoded" % (rank, len(sections), len(idx)), file=sys.stderr,
              flush=True)
    par = parity_check(ctx, j.out_dev, [int(j.so[t]) for t in idx], sections, idx)
    par["rank"] = rank
    return base, par


def merge_parity(per_rank, world):
    """rank 0's parity entry of the line: the ranks' samples summed"""
    return {"checked_channel_blocks": sum(p["checked_channel_blocks"] for p in per_rank),
            "mismatching": sum(p["mismatching"] for p in per_rank),
            "streams_checked": sum(len(p["streams"]) for p in per_rank),
            "ranks": [{"rank": p["rank"], "streams": p["streams"], "checked_channel_blocks":
                       p["checked_channel_blocks"], "mismatching": p["mismatching"],
                       "mismatching_streams": p["mismatching_streams"]} for p in per_rank],
            "against": "oracle/pac_oracle.c on the host: every rank re-encodes whole streams of its own shard "
                       "(stream indices are per rank, into its own job) and compares channel-blocks; %d rank(s)"
                       % world}


class Job:
    """One pac_encode_streams call: streams sharing (sample rate, channels)
    with their PCM resident in HBM."""

    def __init__(self, ctx, p, fo, pcm_dev):
        self.ctx, self.p, self.fo, self.pcm_dev = ctx, p, fo, pcm_dev
        self.ns = len(fo) - 1
        self.bcounts = [shard.blocks_of(int(fo[i + 1] - fo[i])) for i in range(self.ns)]
        self.blocks = int(sum(self.bcounts))
        # the worst case (pac_encode_bound: 6 KB per master channel-block) would
        # be 120 GB at 10^7 blocks; 1 KB per channel-block is > 3x the real
        # average, and the library refuses (PAC_E_CAPACITY), never overflows
        bound = int(ctx.L.pac_encode_bound(C.byref(p), self.ns, fo.ctypes.data_as(C.POINTER(C.c_int64))))
        self.cap = min(bound, self.blocks * p.n_channels * 1024)
        self.out_dev = ctx.alloc(self.cap)
        self.so = None

    def run(self):
        _, self.so = self.ctx.encode_streams(self.p, self.pcm_dev, self.fo, out=self.out_dev,
                                             out_capacity=self.cap, pcm_is_device=True, out_is_device=True)
        return self.ctx.last_timing()

    def free(self):
        self.ctx.free(self.out_dev)
        self.ctx.free(self.pcm_dev)

    def cpu_samples(self, idx, max_frames=4096 * 1024):
        """int16 frames of the streams idx (copied back from HBM)"""
        out = []
        for t in idx:
            n = min(int(self.fo[t + 1] - self.fo[t]), max_frames)
            pcm = np.empty((n, 2), dtype=np.int16)
            self.ctx.to_host(pcm, self.pcm_dev + int(self.fo[t]) * 4)
            out.append(pcm)
        return out


class WavJob(Job):
    """config 3: WAV files (raw bytes, back to back) resident in HBM; one step
    = pac_encode_wav: the header scan, the frame gather and the encoder, all
    on the device (the reference driver's whole encode half)."""

    def __init__(self, ctx, p, blobs, frames_host):
        self.ctx, self.p = ctx, p
        self.ns = len(blobs)
        self.foff = np.zeros(self.ns + 1, dtype=np.int64)
        self.foff[1:] = np.cumsum([len(b) for b in blobs])
        self.blob_dev = ctx.alloc(int(self.foff[-1]) + 8)
        for j, b in enumerate(blobs):        # upload file by file (no host copy of the whole batch)
            ctx.to_device(self.blob_dev + int(self.foff[j]), np.frombuffer(b, dtype=np.uint8))
        info = ctx.wav_scan(self.blob_dev, self.foff, blob_is_device=True)
        self.bcounts = [shard.blocks_of(w.frames) for w in info]
        self.blocks = int(sum(self.bcounts))
        self.frames_host = frames_host
        self.cap = self.blocks * p.n_channels * 1024
        self.out_dev = ctx.alloc(self.cap)
        self.so = None
        self.pcm_dev = None

    def run(self):
        _, self.so, _ = self.ctx.encode_wav(self.p, self.blob_dev, self.foff, blob_is_device=True, out=self.out_dev,
                                            out_capacity=self.cap, out_is_device=True)
        return self.ctx.last_timing()

    def free(self):
        self.ctx.free(self.out_dev)
        self.ctx.free(self.blob_dev)

    def cpu_samples(self, idx, max_frames=4096 * 1024):
        return [self.frames_host[t][:max_frames] for t in idx]


def synthetic_job(a, ctx, rank):
    fs = a.sample_rate
    fps = (a.blocks_per_stream - 1) * 1024
    n_frames = a.streams * fps
    fo = np.arange(a.streams + 1, dtype=np.int64) * fps
    p = _lib.params(fs, 2, 1 if a.master else 0, block_switch=a.bs)
    pcm_dev = ctx.alloc(n_frames * 2 * 2)
    if a.master:
        ctx.synth_pink_tones(pcm_dev, n_frames, fs, seed=1234 + 7919 * rank)
        if a.bs:
            ctx.synth_bursts(pcm_dev, n_frames, 8192, seed=99 + 7919 * rank)
    else:
        ctx.synth_white(pcm_dev, n_frames * 2, seed=1234 + 7919 * rank)
    return [Job(ctx, p, fo, pcm_dev)]


def file_jobs(a, ctx, rank, world):
    """config 3: the stereo inputs x copies as independent streams, this
    rank's LPT shard (pac_amd.shard.plan), one WavJob per sample rate: the raw
    WAV files go to HBM, the parsing happens in the timed step on the device."""
    from pac_amd.pcmfile import read_for_encode
    paths = sorted(glob.glob(os.path.join(INPUTS, "*.wav")))
    reads = [(os.path.basename(pth), pth, *read_for_encode(pth)) for pth in paths]
    stereo = [r for r in reads if r[2].nChannels == 2]
    streams = [(i, c) for i in range(len(stereo)) for c in range(a.copies)]
    counts = [shard.blocks_of(stereo[i][3].shape[0]) for i, _ in streams]
    mine = shard.plan(counts, world)[rank]
    by_fs = {}
    for k in mine:
        i, _ = streams[k]
        by_fs.setdefault(stereo[i][2].sampleRate, []).append(i)
    raw = [open(r[1], "rb").read() for r in stereo]
    jobs = []
    for fs, files in sorted(by_fs.items()):
        jobs.append(WavJob(ctx, _lib.params(fs, 2, 1), [raw[i] for i in files], [stereo[i][3] for i in files]))
    desc = {"inputs": ["%s (%d Hz, %d frames)" % (n, cp.sampleRate, fr.shape[0]) for n, _, cp, fr in stereo],
            "skipped_mono": [n for n, _, cp, _ in reads if cp.nChannels != 2],
            "copies": a.copies, "streams_total": len(streams), "streams_this_rank": len(mine),
            "ingest": "raw WAV bytes in HBM; header scan + frame gather + encode per step (pac_encode_wav)"}
    return jobs, desc, stereo


def bench_decode(a, dist, ctx, job):
    """Decoder throughput: the workload's bitstream (encoded once on the GPU,
    untimed) decoded by pac_decode_streams with input and output in HBM."""
    job.run()
    so = job.so
    frames = job.blocks * 1024
    pcm_out = ctx.alloc(frames * 2 * 2)
    p = job.p

    def step():
        return ctx.decode_streams(p, job.out_dev, so, data_is_device=True, out=pcm_out,
                                  out_capacity_frames=frames, out_is_device=True)

    for _ in range(a.warmup):
        step()
    parse_ms, synth_ms = [], []
    dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        _, fo, _ = step()
        t = ctx.last_timing()
        parse_ms.append(t.front_ms)
        synth_ms.append(t.pack_ms)
    ctx.sync()
    dist.barrier()
    el_max = dist.max(time.perf_counter() - t0)
    total_blocks = dist.sum(job.blocks)
    in_bytes = int(so[-1])
    dec_s = (float(np.mean(parse_ms)) + float(np.mean(synth_ms))) / 1e3
    alg = in_bytes + frames * 4
    res = {
        "metric": "stereo 1024-sample blocks decoded/s",
        "value": total_blocks / (el_max / a.steps),
        "unit": "blocks/s",
        "n_gpus": dist.world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": el_max / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": "synthetic, encoded on the GPU from %s" % ("pink noise + tones" if a.master else "white noise"),
        "config": {"workload": "decode of the configs[%d] workload's bitstream (%d stereo blocks per GPU)"
                               % (a.config, job.blocks),
                   "profile": a.profile, "streams_per_gpu": job.ns, "blocks_per_stream": a.blocks_per_stream,
                   "global_blocks": int(total_blocks),
                   "parallelism": "streams sharded, %d rank(s)" % dist.world},
        "roofline": dec_roofline(alg, dec_s, job.blocks),
        "kernels_ms": {"parse": float(np.mean(parse_ms)), "synth": float(np.mean(synth_ms))},
        "bitstream_bytes_per_gpu": in_bytes,
        "src_hash": _build.source_hash(),
    }
    if dist.rank == 0 and dist.world == 1 and not a.no_cpu:
        res["cpu_baseline"], res["parity"] = cpu_decode(ctx, p, job.out_dev, so, pcm_out, fo, a)
    ctx.free(pcm_out)
    if dist.rank == 0:
        print(json.dumps(res))


def dec_roofline(alg, dec_s, blocks):
    """The decode line's roofline: algorithmic bytes (bitstream read + int16
    PCM written) over the parse + synthesis time of one step, and the PMC HBM
    bytes of the same two kernels (profiles/r*_decode_pmc.json, same source
    hash only) per step."""
    r = {"bound": "hbm", "kernel": "k_dec_parse + k_dec_synth", "achieved": alg / dec_s / 1e9,
         "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": alg / dec_s / 1e9 / HBM_PEAK_GBS, "traffic": None,
         "traffic_unit": "HBM bytes per step (one launch of each kernel: 2 x FETCH_SIZE + WRITE_SIZE)"}
    per_block, srcs = 0.0, []
    for k in ("k_dec_parse", "k_dec_synth"):
        m, src = measured_profile("decode", k)
        if m is None:
            r["traffic_source"] = src
            return r
        per_block += m["hbm_read_bytes_per_block"] + m["hbm_write_bytes_per_block"]
        srcs.append(src)
    r.update({"traffic": per_block * blocks, "traffic_per_block": per_block,
              "traffic_over_alg": per_block * blocks / alg, "traffic_source": srcs[0]})
    return r


def cpu_decode(ctx, p, out_dev, so, pcm_out, fo, a):
    """The oracle's decoder on the first streams' bytes (one host thread per
    stream, bounded), and its frames against the GPU's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as P
    from concurrent.futures import ThreadPoolExecutor
    P.lib()
    threads = max(1, min(a.cpu_threads, len(so) - 1))
    secs = []
    for t in range(threads):
        b = np.empty(int(so[t + 1] - so[t]), dtype=np.uint8)
        ctx.to_host(b, out_dev + int(so[t]))
        secs.append(b.tobytes())
    t0 = time.perf_counter()

    def work(t):
        o = P.Oracle(p.sample_rate, huffman=a.master)
        n = 0
        ref = None
        while time.perf_counter() - t0 < a.cpu_seconds or ref is None:
            ref = o.decode_data(P.MASTER if a.master else P.ORIGIN, secs[t], 2)
            n += ref.shape[0] // 1024
        return n, ref

    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(work, range(threads)))
    el = time.perf_counter() - t0
    done = sum(r[0] for r in res)
    checked = bad = 0
    for t, (_, ref) in enumerate(res):
        got = np.empty(ref.shape, dtype=np.int16)
        ctx.to_host(got, pcm_out + int(fo[t]) * 4)
        checked += ref.shape[0] // 1024
        bad += int(np.sum(np.any((got != ref).reshape(-1, 1024 * 2), axis=1)))
    base = {"value": done / el, "unit": "blocks/s", "cores": threads, "kind": "port",
            "sample": "oracle/pac_oracle.c decoder, %d host threads (one stream each), %d stereo blocks "
                      "in %.1f s" % (threads, done, el)}
    return base, {"checked_blocks": checked, "mismatching": bad,
                  "against": "oracle/pac_oracle.c decoder on the CPU-baseline sample"}


PHASES = {  # pac_timing field -> kernel, per profile (include/pac_gpu.h)
    "origin": [("front_ms", "k_origin_front"), ("alloc_ms", "k_origin_alloc"), ("scan_ms", "k_scan"),
               ("pack_ms", "k_origin_pack")],
    "master": [("lrms_ms", "k_master_lrms"), ("spec_ms", "k_master_spec"), ("thr_ms", "k_master_thr"),
               ("front_ms", "k_master_front"),
               ("alloc_ms", "k_master_tail"), ("emit_ms", "k_master_emit"),
               ("pack_ms", "k_master_place"), ("scan_ms", "k_scan")],
}
PHASES["bs"] = PHASES["master"] + [("thr_short_ms", "k_master_thr_short")]


def main():
    a = parse()
    world = os.environ.get("WORLD_SIZE")
    if world is None and a.gpus > 1:
        sys.exit(spawn_ranks(a))            # N fresh rank processes, one per GPU
    if world is not None and int(world) != a.gpus:
        print("bench.py: --gpus %d but WORLD_SIZE=%s: launch one rank per GPU with --gpus equal to the number "
              "of ranks" % (a.gpus, world), file=sys.stderr)
        sys.exit(2)
    dist = Dist()
    # one GPU per rank (LOCAL_RANK); PAC_BENCH_SHARE_GPU=1 puts every rank on
    # device 0 -- a rehearsal of the multi-rank path on a one-GPU box only
    share = os.environ.get("PAC_BENCH_SHARE_GPU") == "1"
    dev = 0 if share else dist.local
    ctx = make_context(dev, a.master)
    desc, stereo = None, None
    if a.config == 3:
        jobs, desc, stereo = file_jobs(a, ctx, dist.rank, dist.world)
    else:
        jobs = synthetic_job(a, ctx, dist.rank)
    ctx.set_timing(True)
    if a.mode == "decode":
        bench_decode(a, dist, ctx, jobs[0])
        for j in jobs:
            j.free()
        dist.close()
        return

    def step():
        ms = {f: 0.0 for f, _ in PHASES["bs" if a.bs else a.profile]}
        chunks = repacked = 0
        for j in jobs:
            t = j.run()
            for f in ms:
                ms[f] += getattr(t, f)
            chunks += t.chunks
            repacked += t.repacked
        ms["_chunks"], ms["_repacked"] = chunks, repacked
        return ms

    for _ in range(a.warmup):
        step()
    per = []
    dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        per.append(step())
    ctx.sync()
    dist.barrier()
    el = time.perf_counter() - t0
    el_max = dist.max(el)
    blocks = sum(j.blocks for j in jobs)
    out_bytes = sum(int(j.so[-1]) for j in jobs if j.so is not None)
    total_blocks = dist.sum(blocks)
    value = total_blocks / (el_max / a.steps)

    kern_ms = {k: float(np.mean([p[f] for p in per])) for f, k in PHASES["bs" if a.bs else a.profile]}
    if a.master and kern_ms.get("k_master_lrms") == 0.0 and "k_master_spec" in kern_ms:
        # the default fused LRMS + spectra kernel is timed in the spectra phase
        del kern_ms["k_master_lrms"]
        kern_ms["k_master_lrms_spec"] = kern_ms.pop("k_master_spec")
    # the dominant kernel on the critical path (the master reservoir tail runs on
    # a second stream, overlapped with the next chunk's thresholds)
    dom = max((k for k in kern_ms if k not in ("k_master_tail", "k_master_emit")), key=kern_ms.get)
    dom_s = kern_ms[dom] / 1e3
    step_s = el_max / a.steps
    # algorithmic bytes = PCM read + bitstream written, per block
    alg_per_block = PCM_BYTES_PER_BLOCK + out_bytes / blocks
    # launches of the dominant kernel per step: run_master's chunk count (pac_timing.chunks), checked
    # against the host mirror of its chunk geometry
    launches = int(per[-1]["_chunks"]) if a.master and dom != "k_master_place" else len(jobs)
    if a.master and dom != "k_master_place":
        assert launches == sum(master_launches(j.bcounts, chunk_blocks_of(a.bs)) for j in jobs), launches
    achieved = alg_per_block * blocks / dom_s / 1e9 if dom_s > 0 else 0.0
    prof, prof_note = measured_profile("bs" if a.bs else a.profile, dom)   # counters are per workload
    traffic_pb = None
    ref_flop = REF_ALG_FLOP_PER_BLOCK[a.profile]
    fp64 = {"peak_tflops": FP64_PEAK_TFLOPS, "profile": prof_note}
    ref_equiv = {"not_a_roofline": True,
                 "ref_alg_flop_per_block": ref_flop,
                 "ref_alg_equiv_tflops": ref_flop * blocks / step_s / 1e12 if step_s else None,
                 "note": "the reference's direct masking sum priced at ~35 FP64 flop per (masker, line) pair "
                         "(SURVEY 8(d)) at this line's block rate: what the reference ALGORITHM would need, not "
                         "flops executed here (the kernels evaluate factored sums; executed flops: fp64)"}
    if prof:
        if "hbm_read_bytes_per_block" in prof:
            traffic_pb = prof["hbm_read_bytes_per_block"] + prof["hbm_write_bytes_per_block"]
        if "fp64_flop_per_block" in prof and dom_s > 0:
            tf = prof["fp64_flop_per_block"] * blocks / dom_s / 1e12
            fp64.update({"kernel": dom, "executed_flop_per_block": prof["fp64_flop_per_block"],
                         "executed_tflops": tf, "executed_frac": tf / FP64_PEAK_TFLOPS})
        for k in ("valu_issue_util", "fp64_share_of_valu", "lds_bank_conflict_frac"):
            if k in prof:
                fp64[k] = prof[k]
    roofline = {
        "bound": "hbm", "kernel": dom, "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": achieved / HBM_PEAK_GBS,
        "traffic": traffic_pb * blocks / launches if traffic_pb is not None else None,
        "alg_bytes_per_block": alg_per_block,
        "alg_bytes_def": "SURVEY.md 8(d): 4096 B int16 PCM read + the measured bitstream bytes written "
                         "(out_bytes_per_gpu / blocks_per_gpu)",
        "launches_per_step": launches, "blocks_per_launch": blocks / launches,
        "alg_bytes_per_launch": alg_per_block * blocks / launches,
        "avg_launch_ms": kern_ms[dom] / launches,
        "traffic_unit": "HBM bytes per launch (2 x FETCH_SIZE + WRITE_SIZE, profiles/summarize_pmc.py), "
                        "same source hash only",
        "traffic_calibration": "profiles/r06_fetch_calibration.json (tools/probe/fetch_calib.hip): FETCH_SIZE "
                               "counts half the bytes of this kernel's read shapes (8 B per lane: x2.00; 4 x 16 B "
                               "per lane: x1.99), WRITE_SIZE the bytes of its 8 B-per-lane stores exactly -- so "
                               "traffic is a measurement (Infinity Cache hits included), not a bound",
        "traffic_per_block": traffic_pb,
        "traffic_over_alg": traffic_pb / alg_per_block if traffic_pb is not None else None,
        "traffic_source": prof_note,
        "kernel_io_bytes_per_block": KERNEL_IO_BYTES.get(dom),
        "kernel_io_def": "what this kernel of our split reads + writes per block, intermediates included "
                         "(not algorithmic)",
        "step": {"achieved": alg_per_block * blocks / step_s / 1e9,
                 "frac": alg_per_block * blocks / step_s / 1e9 / HBM_PEAK_GBS},
        "binding": binding(dom, prof),
    }
    if a.config == 2:
        data = "synthetic (device-generated pink noise (Voss, counter hash) + 440/1250/5300 Hz tones)"
        workload = ("BASELINE configs[2]: synthetic 48 kHz stereo pink noise + tones, %d stereo blocks per GPU "
                    "(%d streams x %d blocks), N=1024 MDCT, full psychoacoustics + M/S + bit allocation + "
                    "Huffman (master profile)" % (blocks, a.streams, a.blocks_per_stream))
    elif a.config == 4:
        data = ("synthetic (device-generated pink noise + 440/1250/5300 Hz tones + one decaying "
                "gaussian noise burst per 8192 frames at a hashed onset)")
        workload = ("BASELINE configs[4]: block switching N=1024/256 with attack detection (extension, parity "
                    "unpinned: byte-exact vs the oracle's restatement), synthetic 48 kHz stereo, %d stereo "
                    "blocks per GPU (%d streams x %d blocks; 10^8 at 8 GPUs), master profile"
                    % (blocks, a.streams, a.blocks_per_stream))
    elif a.config == 1:
        data = "synthetic (device-generated white noise, counter-hash Box-Muller)"
        workload = ("BASELINE configs[1]: synthetic 48 kHz stereo white noise, %d stereo blocks per GPU "
                    "(%d streams x %d blocks), N=1024 MDCT, M/S off (origin profile)"
                    % (blocks, a.streams, a.blocks_per_stream))
    else:
        data = "real audio: the reference's inputs/*.wav (stereo), tiled as independent streams"
        workload = ("BASELINE configs[3]: %d stereo inputs/*.wav x %d copies, each copy an independent "
                    "master+Huffman stream, LPT-sharded over %d rank(s); %d stereo blocks on rank 0"
                    % (len(stereo), a.copies, dist.world, blocks))
    res = {
        "metric": "stereo 1024-sample blocks encoded/s",
        "value": value,
        "unit": "blocks/s",
        "n_gpus": dist.world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": el_max / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "strong" if a.config == 3 else "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": data,
        "config": {"workload": workload, "profile": a.profile, "global_blocks": int(total_blocks),
                   "blocks_per_gpu": blocks, "parallelism": "streams sharded, %d rank(s), no collective"
                   % dist.world, "tail_mode": os.environ.get("PAC_TAIL_MODE", "overlap")},
        "roofline": roofline,
        "fp64": fp64,
        "ref_alg_equivalent": ref_equiv,
        "kernels_ms": kern_ms,
        "occupancy": occupancy("bs" if a.bs else a.profile, [dom] + [k for k in OCC_KERNELS if k in kern_ms and k != dom]),
        "out_bytes_per_gpu": out_bytes,
        "staging_repacked_calls": int(sum(p["_repacked"] for p in per)),
        "src_hash": _build.source_hash(),
    }
    if desc:
        res["config"]["files"] = desc
    else:
        res["config"].update({"sample_rate": a.sample_rate, "streams_per_gpu": a.streams,
                              "blocks_per_stream": a.blocks_per_stream})
    if not a.no_cpu:
        # every rank checks whole streams of its own shard against the CPU
        # oracle (copied back from HBM, after the timed region); rank 0 reports
        # the sum.  The CPU baseline is rank 0's, timed while the other ranks
        # wait (rank_parity), on rank 0's own host-core share.
        base, par = rank_parity(a, ctx, jobs[0], dist.rank, dist.world, a.cpu_threads,
                                dist=dist if dist.world > 1 else None)
        per_rank = dist.gather(par)
        if dist.rank == 0:
            res["parity"] = merge_parity(per_rank, dist.world)
            base["cpu_share"] = cpu_share()
            if dist.world > 1:
                base["timed_on"] = ("rank 0 of %d, alone (the other ranks wait at a barrier); cores = rank 0's "
                                    "host threads" % dist.world)
            res["cpu_baseline"] = base
    if os.environ.get("PAC_BENCH_MOCK_CONTEXT"):
        res["mock_context"] = "TEST ONLY (%s): no GPU ran, not a measurement" % os.environ["PAC_BENCH_MOCK_CONTEXT"]
    if share and dist.world > 1:
        res["config"]["shared_gpu"] = "PAC_BENCH_SHARE_GPU=1: all %d ranks on device 0 (rehearsal)" % dist.world
    for j in jobs:
        j.free()
    if dist.rank == 0:
        print(json.dumps(res))
    dist.close()


if __name__ == "__main__":
    main()
