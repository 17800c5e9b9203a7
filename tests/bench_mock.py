"""TEST ONLY: a CPU stand-in for pac_amd._lib.Context, loaded by bench.py when
PAC_BENCH_MOCK_CONTEXT names this file (bench.make_context).

It lets tests/test_host.py run `bench.py --gpus 2` end to end on a CPU-only
container: the rank spawn, the gloo barrier / max / sum, every rank's parity
sample and rank 0's line.  "Device memory" is host numpy arrays behind fake
addresses; "encoding" is the CPU oracle (oracle/pyoracle.py), so the parity
sample matches by construction, except where PAC_MOCK_CORRUPT_RANK names the
rank whose first stream gets one byte flipped.  Nothing here is a product
path: bench.py stamps a line made with it "mock_context".
"""
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as P  # noqa: E402
from pac_amd import shard, synth  # noqa: E402

TIMING_FIELDS = ["front_ms", "alloc_ms", "scan_ms", "pack_ms", "total_ms", "thr_ms", "lrms_ms", "thr_short_ms",
                 "spec_ms", "emit_ms"]


def run_master_chunks(nb, chunk_blocks):
    """run_master's launch count (pac_abi.hip), restated for the stand-in"""
    n = 0
    for g0 in range(0, len(nb), chunk_blocks):
        grp = sorted(nb[g0:g0 + chunk_blocks], reverse=True)
        gmax, n_act, t0 = max(1, grp[0]), len(grp), 0
        while t0 < gmax:
            while n_act > 1 and grp[n_act - 1] <= t0:
                n_act -= 1
            t0 += max(1, min(chunk_blocks // n_act, gmax - t0))
            n += 1
    return n


class _L:
    @staticmethod
    def pac_encode_bound(p, ns, fo_p):
        frames = fo_p[ns] - fo_p[0]
        return int((frames // 1024 + 2 * ns) * 2 * 6144)


class Context:
    def __init__(self, device=0, huffman=True):
        self.device, self.huffman = device, huffman
        self.rank = int(os.environ.get("RANK", "0"))
        self.mem = {}
        self.next = 1 << 32
        self.L = _L()
        self.chunks = 0

    def _at(self, addr, nbytes):
        for base, buf in self.mem.items():
            if base <= addr and addr + nbytes <= base + buf.nbytes:
                return buf[addr - base:addr - base + nbytes]
        raise ValueError("mock: bad address %#x (+%d)" % (addr, nbytes))

    def alloc(self, nbytes):
        base = self.next
        self.mem[base] = np.zeros(max(int(nbytes), 1), dtype=np.uint8)
        self.next += (int(nbytes) + 4095) // 4096 * 4096 + 4096
        return base

    def free(self, ptr):
        del self.mem[ptr]

    def to_host(self, arr, src):
        arr.reshape(-1).view(np.uint8)[:] = self._at(src, arr.nbytes)
        return arr

    def to_device(self, dst, arr):
        arr = np.ascontiguousarray(arr)
        self._at(dst, arr.nbytes)[:] = arr.reshape(-1).view(np.uint8)

    def synth_pink_tones(self, dev, n_frames, fs, seed):
        self.to_device(dev, synth.pink_tones_pcm(int(n_frames), fs, seed=int(seed) % (1 << 31)))

    def synth_bursts(self, dev, n_frames, period, seed):
        pass

    def synth_white(self, dev, n_samples, seed):
        self.to_device(dev, synth.white_pcm(int(n_samples) // 2, 2, seed=int(seed) % (1 << 31)))

    def encode_streams(self, p, pcm, fo, out=None, out_capacity=None, pcm_is_device=True, out_is_device=True,
                       states=None):
        prof = P.MASTER if p.profile == 1 else P.ORIGIN
        o = P.Oracle(p.sample_rate, huffman=prof == P.MASTER, block_switch=bool(p.block_switch))
        so = np.zeros(len(fo), dtype=np.int64)
        secs = []
        for i in range(len(fo) - 1):
            n = int(fo[i + 1] - fo[i])
            x = np.empty((n, p.n_channels), dtype=np.int16)
            self.to_host(x, pcm + int(fo[i]) * 2 * p.n_channels)
            secs.append(o.encode_data(prof, x))
            so[i + 1] = so[i] + len(secs[-1])
        buf = np.frombuffer(b"".join(secs), dtype=np.uint8).copy()
        if os.environ.get("PAC_MOCK_CORRUPT_RANK") == str(self.rank) and len(secs[0]) > 9:
            buf[9] ^= 0x10
        assert so[-1] <= out_capacity
        self.to_device(out, buf)
        nb = [shard.blocks_of(int(fo[i + 1] - fo[i])) for i in range(len(fo) - 1)]
        env = os.environ.get("PAC_CHUNK_BLOCKS", "")
        self.chunks = run_master_chunks(nb, int(env) if env.isdigit() else (65536 if p.block_switch else 32768))
        return out, so

    def last_timing(self):
        t = types.SimpleNamespace(**{f: 0.0 for f in TIMING_FIELDS})
        t.chunks, t.repacked = self.chunks, 0
        return t

    def set_timing(self, on):
        pass

    def sync(self):
        pass

    def close(self):
        pass
