#!/usr/bin/env python3
"""Benchmark: stereo 1024-sample blocks encoded per second on MI355X.

Workload (BASELINE.json configs[1], the config the metric is quoted on):
synthetic 48 kHz stereo white noise, N(0,1)*0.25*32767 rounded/clipped to
int16, 10^6 stereo blocks per GPU (1000 independent streams x 1000 blocks,
999 hops + the Close() flush block each), origin profile ("M/S off":
PerceptualAudioCodec_Origin's coder, the reference's own no-M/S encoder).
The PCM is generated on the device (k_synth_white) so the timed region starts
with the inputs resident in HBM; one step = one pac_encode_streams call over
all 10^6 blocks (MDCT, masking threshold, bit allocation, quantization, bit
packing into the .pac data sections, all in HBM).

    python bench.py [--gpus N --steps K --warmup W]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one rank per GPU)

Streams shard across ranks with no data-path collective (weak scaling); the
only cross-rank traffic is the barrier and the max-over-ranks of the timer
(gloo, CPU tensors).  Rank 0 prints one JSON line.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

import pac_amd  # noqa: E402,F401
from pac_amd import _lib  # noqa: E402

HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md chip table (spec)
FP64_PEAK_TFLOPS = 78.6        # MI355X FP64 vector peak (spec)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--mode", choices=["encode", "decode"], default="encode",
                    help="encode = the metric (default); decode = pac_decode_streams of the same "
                         "workload's bitstream (encoded once, untimed)")
    ap.add_argument("--profile", choices=["origin", "master"], default="origin",
                    help="origin = BASELINE configs[1] (white noise, M/S off, the metric's config); "
                         "master = configs[2] (pink noise + tones, M/S + Huffman)")
    ap.add_argument("--streams", type=int, default=None,
                    help="default 1000 (origin, 10^6 blocks) / 10000 (master, 10^7 blocks)")
    ap.add_argument("--blocks-per-stream", type=int, default=1000)
    ap.add_argument("--sample-rate", type=int, default=48000)
    ap.add_argument("--cpu-seconds", type=float, default=12.0,
                    help="bounded CPU-baseline sample (oracle on host cores)")
    ap.add_argument("--cpu-threads", type=int, default=16,
                    help="host threads of the CPU baseline (the GPU box's CPU share is 16)")
    ap.add_argument("--no-cpu", action="store_true")
    a = ap.parse_args()
    if a.streams is None:
        a.streams = 10000 if a.profile == "master" else 1000
    return a


class Dist:
    """Barrier + max over ranks; gloo on CPU when launched under torchrun."""

    def __init__(self):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.td = None
        if self.world > 1:
            import torch.distributed as td
            td.init_process_group("gloo")
            self.td = td

    def barrier(self):
        if self.td:
            self.td.barrier()

    def max(self, v):
        if not self.td:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.td.all_reduce(t, op=self.td.ReduceOp.MAX)
        return float(t.item())

    def sum(self, v):
        if not self.td:
            return v
        import torch
        t = torch.tensor([float(v)], dtype=torch.float64)
        self.td.all_reduce(t, op=self.td.ReduceOp.SUM)
        return float(t.item())

    def close(self):
        if self.td:
            self.td.destroy_process_group()


# the reference's direct masking sum costs ~35 FP64
# flops per (masker, line) pair, ~2 x 255 x 1024 pairs per stereo block for
# the origin coder -> ~18 MFLOP per block.  Our kernel evaluates the same sum
# in factored forms; "ref_alg_equiv_tflops" prices our rate at
# the reference algorithm's flop count.
REF_ALG_FLOP_PER_BLOCK = 18.0e6
REF_ALG_FLOP_PER_BLOCK_MASTER = 48.0e6     # 6 thresholds x ~222 maskers x 1024 lines


def measured_profile():
    """Per-block HBM bytes and FP64 work of k_origin_front from the newest
    committed rocprofv3 PMC summary (profiles/*_origin_pmc.json, made by
    profiles/run_profile.sh + profiles/summarize_pmc.py on this kernel build)."""
    import glob
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "r*_origin_pmc.json")))
    if not files:
        return None
    with open(files[-1]) as f:
        d = json.load(f)
    if "k_origin_front" not in d:
        return None
    d["_file"] = os.path.relpath(files[-1], ROOT)
    return d


def cpu_baseline(ctx, dev_pcm, frames_per_stream, n_streams, fs, seconds, profile, threads):
    """The CPU oracle (oracle/pac_oracle.c) on a bounded sample of the same
    workload, one host thread per stream (ctypes releases the GIL; the C
    oracle keeps no global state): thread t encodes growing prefixes of stream
    t, copied back from HBM, until `seconds` have passed."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as P
    from concurrent.futures import ThreadPoolExecutor
    P.lib()
    threads = max(1, min(threads, n_streams))
    hops = min(frames_per_stream // 1024, 4096)
    pcms = []
    for t in range(threads):
        pcm = np.empty((hops * 1024, 2), dtype=np.int16)
        ctx.to_host(pcm, dev_pcm + t * frames_per_stream * 4)
        pcms.append(pcm)
    prof = P.MASTER if profile == "master" else P.ORIGIN
    t0 = time.perf_counter()

    def work(t):
        o = P.Oracle(fs, huffman=(prof == P.MASTER))
        done, chunk, last = 0, 16, b""
        while time.perf_counter() - t0 < seconds and done < 200000:
            n = min(chunk, hops - 1)
            last = o.encode_data(prof, pcms[t][: n * 1024], max_blocks=n)
            done += n
            chunk = min(chunk * 2, hops - 1)
        return done, last

    with ThreadPoolExecutor(threads) as ex:
        res = list(ex.map(work, range(threads)))
    el = time.perf_counter() - t0
    done = sum(r[0] for r in res)
    base = {"value": done / el, "unit": "blocks/s", "cores": threads, "kind": "port",
            "sample": "oracle/pac_oracle.c (C restatement, byte-exact on the 16 reference "
                      "fixtures), %s profile, %d host threads (one stream each), %d stereo "
                      "blocks of the same synthetic streams in %.1f s" % (profile, threads, done, el)}
    return base, [r[1] for r in res]


def channel_blocks(b):
    """split a data section into its '<L nBytes' + payload channel-blocks"""
    out, pos = [], 0
    while pos + 4 <= len(b):
        n = int.from_bytes(b[pos:pos + 4], "little")
        out.append(b[pos:pos + 4 + n])
        pos += 4 + n
    return out


def parity_check(ctx, out_dev, so, oracle_prefixes):
    """The oracle's bytes for the first blocks of streams 0..T-1 (from the CPU
    baseline run) against the GPU's bytes for the same streams: the number of
    channel-blocks compared and how many differ (flip rate)."""
    checked = bad = 0
    for t, ref in enumerate(oracle_prefixes):
        if not ref:
            continue
        got = np.empty(len(ref), dtype=np.uint8)
        ctx.to_host(got, out_dev + int(so[t]))
        a, b = channel_blocks(ref), channel_blocks(got.tobytes())
        checked += len(a)
        bad += sum(1 for x, y in zip(a, b) if x != y) + max(0, len(a) - len(b))
    return {"checked_channel_blocks": checked, "mismatching": bad,
            "against": "oracle/pac_oracle.c on the CPU-baseline sample"}


def bench_decode(a, dist, ctx, p, encode_step, out_dev, ns, blocks, master):
    """Decoder throughput: the workload's bitstream (encoded once on the GPU,
    untimed) decoded by pac_decode_streams with input and output in HBM."""
    _, so = encode_step()
    frames = blocks * 1024
    pcm_out = ctx.alloc(frames * 2 * 2)

    def step():
        return ctx.decode_streams(p, out_dev, so, data_is_device=True, out=pcm_out,
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
    total_blocks = dist.sum(blocks)
    in_bytes = int(so[-1])
    # algorithmic bytes per launch of the decode path: the bitstream read once
    # + int16 PCM written once
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
        "data": "synthetic, encoded on the GPU from %s" % ("pink noise + tones" if master else "white noise"),
        "config": {"workload": "decode of the %s workload's bitstream (%d stereo blocks per GPU)"
                               % ("configs[2]" if master else "configs[1]", blocks),
                   "profile": a.profile, "streams_per_gpu": ns, "blocks_per_stream": a.blocks_per_stream,
                   "global_blocks": int(total_blocks),
                   "parallelism": "streams sharded, %d rank(s)" % dist.world},
        "roofline": {"bound": "hbm", "kernel": "k_dec_parse + k_dec_synth", "achieved": alg / dec_s / 1e9,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": alg / dec_s / 1e9 / HBM_PEAK_GBS,
                     "traffic": None},
        "kernels_ms": {"parse": float(np.mean(parse_ms)), "synth": float(np.mean(synth_ms))},
        "bitstream_bytes_per_gpu": in_bytes,
    }
    if dist.rank == 0 and dist.world == 1 and not a.no_cpu:
        res["cpu_baseline"], res["parity"] = cpu_decode(ctx, p, out_dev, so, pcm_out, fo, a, master)
    ctx.free(pcm_out)
    if dist.rank == 0:
        print(json.dumps(res))
    dist.close()


def cpu_decode(ctx, p, out_dev, so, pcm_out, fo, a, master):
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
        o = P.Oracle(a.sample_rate, huffman=master)
        n = 0
        ref = None
        while time.perf_counter() - t0 < a.cpu_seconds or ref is None:
            ref = o.decode_data(P.MASTER if master else P.ORIGIN, secs[t], 2)
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


def main():
    a = parse()
    dist = Dist()
    master = a.profile == "master"
    ctx = _lib.Context(dist.local, huffman=master)
    fs = a.sample_rate
    hops = a.blocks_per_stream - 1
    fps = hops * 1024
    ns = a.streams
    n_frames = ns * fps
    fo = np.arange(ns + 1, dtype=np.int64) * fps
    p = _lib.params(fs, 2, 1 if master else 0)
    blocks = ns * a.blocks_per_stream
    pcm_dev = ctx.alloc(n_frames * 2 * 2)
    if master:
        ctx.synth_pink_tones(pcm_dev, n_frames, fs, seed=1234 + 7919 * dist.rank)
    else:
        ctx.synth_white(pcm_dev, n_frames * 2, seed=1234 + 7919 * dist.rank)
    cap = int(ctx.L.pac_encode_bound(C.byref(p), ns, fo.ctypes.data_as(C.POINTER(C.c_int64))))
    out_dev = ctx.alloc(cap)
    ctx.set_timing(True)

    def step():
        return ctx.encode_streams(p, pcm_dev, fo, out=out_dev, out_capacity=cap,
                                  pcm_is_device=True, out_is_device=True)

    if a.mode == "decode":
        return bench_decode(a, dist, ctx, p, step, out_dev, ns, blocks, master)

    for _ in range(a.warmup):
        step()
    fronts, alloc_ms, pack_ms, totals = [], [], [], []
    dist.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    for _ in range(a.steps):
        _, so = step()
        t = ctx.last_timing()
        fronts.append(t.front_ms)
        alloc_ms.append(t.alloc_ms)
        pack_ms.append(t.pack_ms)
        totals.append(t.total_ms)
    ctx.sync()
    dist.barrier()
    el = time.perf_counter() - t0
    el_max = dist.max(el)
    out_bytes = int(so[-1])
    total_blocks = dist.sum(blocks)
    value = total_blocks / (el_max / a.steps)

    # roofline of the dominant kernel.  origin: k_origin_front, algorithmic
    # bytes per launch = int16 PCM read (4096 B per stereo block) + SMR/peak/
    # scale outputs (2 x (25*8 + 25*8 + 1) B per stereo block).  master: the
    # front time covers k_master_thr + k_master_front; k_master_thr reads the
    # PCM (4096 B) and writes the 6 thresholds (6 x 1024 x 8 B) per block.
    front_s = float(np.mean(fronts)) / 1e3
    kern = "k_master_thr" if master else "k_origin_front"
    per_block = 4096 + (6 * 1024 * 8 if master else 2 * (25 * 8 * 2 + 1))
    alg_bytes = blocks * per_block
    achieved = alg_bytes / front_s / 1e9
    prof = None if master else measured_profile()
    traffic = None
    ref_flop = REF_ALG_FLOP_PER_BLOCK_MASTER if master else REF_ALG_FLOP_PER_BLOCK
    fp64 = {"ref_alg_flop_per_block": ref_flop,
            "ref_alg_equiv_tflops": ref_flop * blocks / front_s / 1e12,
            "peak_tflops": FP64_PEAK_TFLOPS}
    if prof:
        f = prof["k_origin_front"]
        traffic = (f["hbm_read_bytes_per_block"] + f["hbm_write_bytes_per_block"]) * blocks
        fp64.update({"executed_flop_per_block": f["fp64_flop_per_block"],
                     "executed_tflops": f["fp64_flop_per_block"] * blocks / front_s / 1e12,
                     "executed_frac": f["fp64_flop_per_block"] * blocks / front_s / 1e12 / FP64_PEAK_TFLOPS,
                     "valu_issue_util": f["valu_issue_util"], "source": prof["_file"]})
    if master:
        data = "synthetic (device-generated pink noise (Voss, counter hash) + 440/1250/5300 Hz tones)"
        workload = ("BASELINE configs[2]: synthetic 48 kHz stereo pink noise + tones, %d stereo "
                    "blocks per GPU, N=1024 MDCT, full psychoacoustics + M/S + bit allocation + "
                    "Huffman (master profile)" % blocks)
    else:
        data = "synthetic (device-generated white noise, counter-hash Box-Muller)"
        workload = ("BASELINE configs[1]: synthetic 48 kHz stereo white noise, 10^6 stereo blocks "
                    "per GPU, N=1024 MDCT, M/S off (origin profile)")
    res = {
        "metric": "stereo 1024-sample blocks encoded/s",
        "value": value,
        "unit": "blocks/s",
        "n_gpus": dist.world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": el_max / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f64",
        "data": data,
        "config": {"workload": workload,
                   "profile": a.profile, "sample_rate": fs, "streams_per_gpu": ns,
                   "blocks_per_stream": a.blocks_per_stream,
                   "global_blocks": int(total_blocks), "parallelism": "streams sharded, %d rank(s)"
                   % dist.world},
        "roofline": {"bound": "hbm", "kernel": kern, "achieved": achieved,
                     "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": achieved / HBM_PEAK_GBS,
                     "traffic": traffic,
                     "traffic_source": prof["_file"] if prof else None,
                     "note": "%s is FP64-VALU bound (masking sum), not HBM bound: "
                             "see 'fp64' and DESIGN.md section 4" % kern},
        "fp64": fp64,
        "kernels_ms": {"front": float(np.mean(fronts)), "alloc": float(np.mean(alloc_ms)),
                       "pack": float(np.mean(pack_ms)), "step_device": float(np.mean(totals))},
        "out_bytes_per_gpu": out_bytes,
    }
    if dist.rank == 0 and dist.world == 1 and not a.no_cpu:
        res["cpu_baseline"], prefixes = cpu_baseline(ctx, pcm_dev, fps, ns, fs, a.cpu_seconds, a.profile,
                                                     a.cpu_threads)
        res["parity"] = parity_check(ctx, out_dev, so, prefixes)
    ctx.free(out_dev)
    ctx.free(pcm_dev)
    if dist.rank == 0:
        print(json.dumps(res))
    dist.close()


if __name__ == "__main__":
    main()
