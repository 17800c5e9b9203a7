"""CPU-only tests of the host side: the C-ABI library loads and exports every
symbol include/pac_gpu.h declares (no compute without a GPU), host mirrors of
the reference's file-format logic, the Huffman table export, the synthetic
generators and the stream shard planner (gloo, world_size 2)."""
import ctypes as C
import json
import os
import re
import struct
import subprocess
import sys

import numpy as np
import pytest

from conftest import GOLD, REF, ROOT, fixture

import pac_amd  # noqa: F401
from pac_amd import _lib, pacfile, pcmfile, psychoac, shard, synth
from pac_amd.huffman import Huffman, load_tables


def header_symbols():
    with open(os.path.join(ROOT, "include", "pac_gpu.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"\b(pac_[a-z_0-9]+)\s*\(", txt)))


def test_library_exports_every_header_symbol():
    L = _lib.lib()
    syms = header_symbols()
    assert len(syms) >= 18
    for s in syms:
        assert hasattr(L, s), s
    assert L.pac_version() >= 100


def test_nm_exports_are_extern_c():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (pac_[a-z_0-9]+)$", out, re.M))
    assert set(header_symbols()) <= exported


def test_no_gpu_errors_are_loud():
    """Without a GPU the context refuses (no silent CPU fallback)."""
    L = _lib.lib()
    h = C.c_void_p()
    rc = L.pac_ctx_create(0, C.byref(h))
    if rc == 0:
        L.pac_ctx_destroy(h)
        pytest.skip("a GPU is present")
    assert rc == -2
    assert b"device" in L.pac_last_error().lower() or b"hip" in L.pac_last_error().lower()


@pytest.mark.parametrize("fs", [8000, 16000, 22050, 32000, 44100, 48000, 96000])
def test_band_layout_host_equals_abi(fs):
    assert psychoac.AssignMDCTLinesFromFreqLimits(1024, fs) == list(_lib.band_layout(fs))
    assert sum(psychoac.AssignMDCTLinesFromFreqLimits(1024, fs)) <= 1024


def test_band_layouts_match_survey():
    assert psychoac.AssignMDCTLinesFromFreqLimits(1024, 44100) == [
        5, 4, 5, 5, 5, 5, 7, 7, 7, 9, 10, 11, 13, 15, 17, 21, 26, 32, 42, 51, 61, 83, 116, 163, 304]
    assert psychoac.AssignMDCTLinesFromFreqLimits(1024, 48000) == [
        4, 5, 4, 4, 5, 5, 6, 6, 7, 8, 9, 10, 12, 14, 16, 19, 24, 30, 38, 47, 56, 76, 107, 149, 363]


def test_header_quirk():
    """pacfile.py:240-242: only exact multiples of 1024 are bumped."""
    h = pacfile.header_bytes(44100, 2, 102400)
    assert struct.unpack("<LHLLHH", h[4:22])[2] == 103424
    h = pacfile.header_bytes(44100, 2, 102401)
    assert struct.unpack("<LHLLHH", h[4:22])[2] == 102401
    with open(fixture("harpsichord.pac"), "rb") as f:
        ref = f.read()
    assert pacfile.header_bytes(44100, 2, 394646) == ref[:len(pacfile.header_bytes(44100, 2, 394646))]


def test_pcm_reader_matches_reference_conversion():
    cp, frames = pcmfile.read_for_encode(fixture("harpsichord.wav"))
    assert (cp.sampleRate, cp.nChannels, cp.numSamples) == (44100, 2, 394646)
    assert frames.shape == (394646, 2)
    x = pcmfile.codes_to_float(np.array([-32768, -32767, -1, 0, 1, 32767]))
    assert np.signbit(x[0]) == False and x[0] == 0.0          # the -32768 quirk
    assert x[1] == -(2.0 * 32767 / 65535.0) and x[5] == 2.0 * 32767 / 65535.0
    assert x[2] == -(2.0 / 65535.0) and x[3] == 0.0


def test_pcmfile_hop_reads_equal_bulk(tmp_path):
    """PCMFile.ReadDataBlock hop by hop == read_for_encode (zero-padded tail)."""
    pcm = synth.white_pcm(3 * 1024 + 5, 2, seed=3)
    p = tmp_path / "x.wav"
    with open(p, "wb") as f:
        d = pcm.astype("<i2").tobytes()
        f.write(struct.pack("<4sL4s4sLHHLLHH4sL", b"RIFF", 36 + len(d), b"WAVE", b"fmt ", 16, 1, 2,
                            48000, 48000 * 4, 4, 16, b"data", len(d)) + d)
    pf = pcmfile.PCMFile(str(p))
    cp = pf.OpenForReading()
    cp.nSamplesPerBlock = 1024
    hops = []
    while True:
        blk = pf.ReadDataBlock(cp)
        if blk is None:
            break
        hops.append(np.stack(blk, 1))
    pf.Close(cp)
    assert len(hops) == 4
    _, frames = pcmfile.read_for_encode(str(p))
    whole = np.concatenate(hops)[: frames.shape[0]]
    assert np.array_equal(whole, pcmfile.codes_to_float(frames))
    assert np.all(np.concatenate(hops)[frames.shape[0]:] == 0)


def _hop_loop(path):
    """the reference driver's reads: PCMFile.ReadDataBlock until None, with
    PACFile.WriteFileHeader's bump of the shared numSamples (pacfile.py:240-242)"""
    pf = pcmfile.PCMFile(str(path))
    cp = pf.OpenForReading()
    cp.nSamplesPerBlock = 1024
    if cp.numSamples % 1024 == 0:
        cp.numSamples += 1024
    hops = []
    while True:
        blk = pf.ReadDataBlock(cp)
        if blk is None:
            break
        hops.append(np.stack(blk, 1))
    pf.Close(cp)
    return hops


@pytest.mark.parametrize("claimed", [3 * 1024 + 5, 4 * 1024, 0xFFFFFFFF // 4])
@pytest.mark.parametrize("cut", [0, 1, 3, 4 * 1024 + 2, 2 * 4096, 3 * 4096 + 7])
def test_truncated_wav_reads_to_last_byte(tmp_path, claimed, cut):
    """a data chunk cut short (or a streaming header's 0xFFFFFFFF): the reads
    stop at the first empty hop, the partial one zero-padded, no extra hop --
    read_for_encode == the hop loop"""
    pcm = synth.white_pcm(4 * 1024, 2, seed=cut)
    d = pcm.astype("<i2").tobytes()[:cut]
    p = tmp_path / "t.wav"
    p.write_bytes(struct.pack("<4sL4s4sLHHLLHH4sL", b"RIFF", 36 + len(d), b"WAVE", b"fmt ", 16, 1, 2,
                              48000, 48000 * 4, 4, 16, b"data", min(claimed * 4, 0xFFFFFFFF)) + d)
    hops = _hop_loop(p)
    _, frames = pcmfile.read_for_encode(str(p))
    assert frames.shape[0] == (cut + 3) // 4
    assert len(hops) == (frames.shape[0] + 1023) // 1024
    if hops:
        whole = np.concatenate(hops)
        assert np.array_equal(whole[: frames.shape[0]], pcmfile.codes_to_float(frames))
        assert np.all(whole[frames.shape[0]:] == 0)


def test_exact_multiple_reads_trailing_chunk(tmp_path):
    """numSamples % 1024 == 0: the bumped header count makes the reference
    reader take one more hop from the bytes after the data chunk."""
    pcm = synth.white_pcm(2 * 1024, 2, seed=4)
    p = tmp_path / "y.wav"
    tail = b"LIST\x04\x00\x00\x00abcd"
    with open(p, "wb") as f:
        d = pcm.astype("<i2").tobytes()
        f.write(struct.pack("<4sL4s4sLHHLLHH4sL", b"RIFF", 36 + len(d) + len(tail), b"WAVE", b"fmt ",
                            16, 1, 2, 48000, 48000 * 4, 4, 16, b"data", len(d)) + d + tail)
    _, frames = pcmfile.read_for_encode(str(p))
    assert frames.shape[0] == 3 * 1024
    assert np.array_equal(frames[:2048], pcm)
    raw = np.frombuffer(tail + b"\0" * (4096 - len(tail)), "<i2").reshape(-1, 2)
    assert np.array_equal(frames[2048:], raw)


def test_float_to_codes_roundtrip():
    c = np.arange(-32767, 32768, 7, dtype=np.int16)
    assert np.array_equal(pcmfile.float_to_codes(pcmfile.codes_to_float(c)), c)


def test_huffman_tables_image():
    t = load_tables()
    assert sorted(t) == list(range(1, 11))
    assert len(t[5]) == 4492 and len(t[8]) == 67
    for tid, enc in t.items():
        codes = sorted(enc.values(), key=len)
        # prefix-free
        s = set()
        for c in codes:
            assert not any(c[:k] in s for k in range(1, len(c) + 1)), (tid, c)
            s.add(c)


@pytest.mark.skipif(not os.path.isdir(REF), reason="reference checkout not present")
def test_huffman_export_matches_pickle_stream():
    """Re-export from the reference pickle (opcode-walk, nothing executed)."""
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import export_huffman_tables as ex
    with open(ex.REF, "rb") as f:
        root = ex.parse_protocol0(f.read())
    t = load_tables()
    for tid in range(1, 11):
        assert root[tid].state["encodingTable"] == t[tid]


def test_huffman_reservoir_semantics():
    """withdrawBits (Huffman.py:363-371) with Python-2 floor division."""
    h = Huffman()
    h.depositBits(1234)
    assert h.withdrawBits() == 12 and h.getBitDeposit() == 1222
    h.bitDeposit = 10
    assert h.withdrawBits() == 0 and h.bitDeposit == 10
    h.bitDeposit = -37
    assert h.withdrawBits() == -37 and h.bitDeposit == 0


def test_hash_white_mirror_is_gaussian():
    x = synth.hash_white_pcm(200000, 1234).astype(np.float64) / (0.25 * 32767)
    assert abs(x.mean()) < 0.01 and abs(x.std() - 1) < 0.01


def test_shard_plan_lpt():
    counts = [1001, 5, 300, 300, 2000, 7, 1001]
    sh = shard.plan(counts, 3)
    assert sorted(i for s in sh for i in s) == list(range(len(counts)))
    loads, imb = shard.balance(counts, sh)
    assert loads.max() == 2000      # the single longest stream bounds the makespan
    assert shard.plan(counts, 1) == [list(range(len(counts)))]
    assert shard.blocks_of(0) == 1 and shard.blocks_of(1024) == 2 and shard.blocks_of(1025) == 3


GLOO_WORKER = r"""
import os, sys
sys.path.insert(0, %r)
import torch.distributed as td
import pac_amd
from pac_amd import shard
td.init_process_group("gloo")
r, w = td.get_rank(), td.get_world_size()
counts = [shard.blocks_of(n) for n in (5000, 1, 40000, 123456, 7777, 1024 * 1000, 3, 99999)]
mine = shard.plan(counts, w)[r]
allp = [None] * w
td.all_gather_object(allp, mine)
flat = sorted(i for p in allp for i in p)
assert flat == list(range(len(counts))), flat
assert all(set(allp[a]).isdisjoint(allp[b]) for a in range(w) for b in range(a + 1, w))
td.barrier()
if r == 0:
    print("GLOO_OK", allp)
td.destroy_process_group()
"""


def test_shard_plan_gloo_world2(tmp_path):
    """The N>1 path: every rank derives the same plan; shards are disjoint and
    cover all streams (gloo all_gather on CPU, world_size 2)."""
    script = tmp_path / "w.py"
    script.write_text(GLOO_WORKER % ROOT)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT="29517")
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port", "29517",
                        str(script)], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert "GLOO_OK" in r.stdout


@pytest.mark.parametrize("n", [0, 1, 1023, 1024, 1025, 5 * 1024, 37 * 1024 + 11])
@pytest.mark.parametrize("parts", [1, 2, 3, 7])
def test_split_stream_plan(n, parts):
    """shard.split_stream: the parts cover every hop exactly once, each later
    part carries the one-hop halo (its priorBlock) and only the last part
    ends with the flush block."""
    from pac_amd import shard, _lib
    sp = shard.split_stream(n, parts)
    hops = (n + 1023) // 1024
    assert 1 <= len(sp) <= max(1, min(parts, hops))
    covered = []
    for i, (lo, hi, fl) in enumerate(sp):
        prior = 1024 if fl & _lib.STREAM_HAS_PRIOR else 0
        assert bool(fl & _lib.STREAM_HAS_PRIOR) == (i > 0)
        assert bool(fl & _lib.STREAM_NO_FLUSH) == (i < len(sp) - 1)
        first = (lo + prior) // 1024
        nh = (max(hi - lo - prior, 0) + 1023) // 1024
        covered += list(range(first, first + nh))
        assert hi <= n and lo >= 0
    assert covered == list(range(hops))


@pytest.mark.parametrize("name,prof", [("piano_test2.wak", 1), ("harpsichord.pac", 0)])
def test_decode_layout_on_host(name, prof):
    """pac_decode_layout (host only, no GPU): the decoded frame count of a
    reference file equals the oracle's decode, and a truncated section is
    refused like the reference's reader refuses it."""
    from pac_amd import _lib
    import pyoracle as P
    with open(fixture(name), "rb") as f:
        b = f.read()
    fs, nch, ns, nl, off = P.parse_pac_header(b)
    data = np.frombuffer(b[off:], dtype=np.uint8)
    so = np.array([0, len(data)], dtype=np.int64)
    fo = np.zeros(2, dtype=np.int64)
    p = _lib.params(fs, nch, prof)
    L = _lib.lib()
    P64 = C.POINTER(C.c_int64)
    assert L.pac_decode_layout(C.byref(p), 1, data.ctypes.data, so.ctypes.data_as(P64), 0, fo.ctypes.data_as(P64)) == 0
    o = P.Oracle(fs, huffman=bool(prof))
    assert int(fo[1]) == o.decode_data(prof, b[off:], nch).shape[0]
    so2 = np.array([0, len(data) - 3], dtype=np.int64)
    assert L.pac_decode_layout(C.byref(p), 1, data.ctypes.data, so2.ctypes.data_as(P64), 0,
                               fo.ctypes.data_as(P64)) == -1


BENCH_DIST_WORKER = r"""
import importlib.util, sys
sys.argv = ["bench.py"]
spec = importlib.util.spec_from_file_location("bench", "%s/bench.py")
b = importlib.util.module_from_spec(spec)
spec.loader.exec_module(b)
d = b.Dist()
d.barrier()
if d.rank == 0:
    print("MAX %%s SUM %%s" %% (d.max(d.rank + 1.5), d.sum(d.rank + 1)))
else:
    d.max(d.rank + 1.5), d.sum(d.rank + 1)
d.close()
"""


def test_bench_dist_gloo_world2(tmp_path):
    """bench.py's multi-rank plumbing (torchrun, gloo barrier, max / sum over
    ranks) at world size 2 on the CPU, and stdout keeps only rank 0's line
    (gloo's connection banner is sent to stderr)."""
    script = tmp_path / "d.py"
    script.write_text(BENCH_DIST_WORKER % ROOT)
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port", "29519",
                        str(script)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    assert r.stdout.strip().splitlines() == ["MAX 2.5 SUM 3.0"]


BENCH_PARITY_WORKER = r"""
import importlib.util, json, sys, types
import numpy as np
sys.argv = ["bench.py"]
sys.path.insert(0, "%s/oracle")
spec = importlib.util.spec_from_file_location("bench", "%s/bench.py")
b = importlib.util.module_from_spec(spec)
spec.loader.exec_module(b)
import pyoracle as P
from pac_amd import synth
d = b.Dist()
fs, ns = 48000, 20
# this rank's streams and the "GPU" bytes: the oracle's own encodes laid out
# back to back in a host buffer standing in for HBM; rank 1 corrupts one byte
# of its stream 5 (a mismatch the parity sample must see and rank 0 report)
pcm = [synth.pink_tones_pcm(1024 * (3 + (i %% 3)) + 77 * i, fs, seed=100 * d.rank + i) for i in range(ns)]
o = P.Oracle(fs, huffman=True)
secs = [o.encode_data(P.MASTER, x) for x in pcm]
so = np.zeros(ns + 1, dtype=np.int64)
so[1:] = np.cumsum([len(x) for x in secs])
hbm = bytearray(b"".join(secs))
if d.rank == 1:
    hbm[int(so[5]) + 9] ^= 0x10
class Ctx:
    def to_host(self, arr, addr):
        arr[:] = np.frombuffer(bytes(hbm[addr:addr + arr.nbytes]), dtype=arr.dtype).reshape(arr.shape)
job = types.SimpleNamespace(ns=ns, so=so, out_dev=0, p=types.SimpleNamespace(sample_rate=fs),
                            cpu_samples=lambda idx: [pcm[t] for t in idx])
a = types.SimpleNamespace(parity_streams=24, profile="master", bs=False, cpu_blocks=-1)
base, par = b.rank_parity(a, Ctx(), job, d.rank, d.world, 4)
allp = d.gather(par)
if d.rank == 0:
    print(json.dumps(b.merge_parity(allp, d.world)))
d.close()
"""


def test_bench_parity_every_rank_gloo_world2(tmp_path):
    """bench.py's N>1 parity: every rank re-encodes whole streams
    of its own shard with the CPU oracle and compares them with its "GPU"
    bytes; rank 0's line carries both ranks' sampled streams and the summed
    mismatches (gloo all_gather_object, world size 2 on the CPU; the GPU
    bytes are stood in by the oracle's own, with one byte of rank 1's stream 5
    flipped)."""
    import json
    script = tmp_path / "p.py"
    script.write_text(BENCH_PARITY_WORKER % (ROOT, ROOT))
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
                        "--nproc-per-node=2", "--master-addr", "127.0.0.1", "--master-port", "29523",
                        str(script)], capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert [x["rank"] for x in line["ranks"]] == [0, 1]
    assert all(len(x["streams"]) == 16 for x in line["ranks"])      # max(16, ceil(24 / 2)), of 20
    assert line["streams_checked"] == 32
    assert line["ranks"][0]["mismatching"] == 0
    assert line["ranks"][1]["mismatching"] == 1 and line["ranks"][1]["mismatching_streams"] == [5]
    assert line["mismatching"] == 1
    assert line["checked_channel_blocks"] == sum(x["checked_channel_blocks"] for x in line["ranks"]) > 32 * 8


def _bench_module():
    import importlib.util
    saved = sys.argv
    sys.argv = ["bench.py"]
    try:
        spec = importlib.util.spec_from_file_location("bench_mod", os.path.join(ROOT, "bench.py"))
        b = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(b)
    finally:
        sys.argv = saved
    return b


def test_bench_parity_sample_spans_the_batch():
    """bench.py's CPU-baseline / parity sample: first and last stream, the
    one-lane tail's wave boundaries, then an even stride."""
    b = _bench_module()
    idx = b.sample_streams(10000, 16)
    assert len(idx) == 16 and idx == sorted(set(idx))
    assert {0, 63, 64, 4095, 4096, 9999} <= set(idx)
    assert max(np.diff(idx)) < 1000
    assert b.sample_streams(22, 16)[-1] == 21 and len(b.sample_streams(22, 16)) == 16
    assert b.sample_streams(3, 16) == [0, 1, 2]


def test_bench_chunk_geometry_mirror(monkeypatch):
    """bench.py mirrors run_master's chunk count (the line's launches_per_step,
    checked against pac_timing.chunks on the GPU): 32768-block chunks, 65536
    with block switching, PAC_CHUNK_BLOCKS overrides."""
    b = _bench_module()
    monkeypatch.delenv("PAC_CHUNK_BLOCKS", raising=False)
    assert b.chunk_blocks_of(False) == 32768 and b.chunk_blocks_of(True) == 65536
    monkeypatch.setenv("PAC_CHUNK_BLOCKS", "7")
    assert b.chunk_blocks_of(True) == 7
    assert b.master_launches([1000] * 10000, 32768) == 334       # S = 3: ceil(1000 / 3)
    assert b.master_launches([1000] * 12500, 65536) == 200       # S = 5
    # ragged: 10, 4, 1 blocks in chunks of 4: S = 1 (3 running), 2, 2 (2 running), 4, 1 (one left)
    assert b.master_launches([10, 4, 1], 4) == 5


def _bench_env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env.update(kw)
    return env


def test_bench_gpus2_spawns_ranks():
    """`bench.py --gpus 2` without torchrun: the parent starts two
    rank processes (gloo), relays rank 0's one JSON line with n_gpus 2, both
    ranks' parity samples and a cpu_baseline.  The HIP context is replaced by
    the CPU stand-in tests/bench_mock.py (the oracle's bytes; rank 1's first
    stream has one byte flipped, which the merged parity must report)."""
    import json
    env = _bench_env(PAC_BENCH_MOCK_CONTEXT=os.path.join(ROOT, "tests", "bench_mock.py"), PAC_MOCK_CORRUPT_RANK="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "2", "--warmup",
                        "1", "--streams", "3", "--blocks-per-stream", "4", "--cpu-threads", "2"],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = r.stdout.strip().splitlines()
    assert len(lines) == 1, r.stdout
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["steps"] == 2 and "mock_context" in line
    assert line["config"]["global_blocks"] == 2 * line["config"]["blocks_per_gpu"] == 2 * 3 * 4
    par = line["parity"]
    assert [x["rank"] for x in par["ranks"]] == [0, 1]
    assert par["ranks"][0]["mismatching"] == 0
    assert par["ranks"][1]["mismatching"] == 1 and par["ranks"][1]["mismatching_streams"] == [0]
    assert par["checked_channel_blocks"] == 2 * 3 * 4 * 2
    base = line["cpu_baseline"]
    assert base["kind"] == "port" and base["cores"] == 2 and "rank 0 of 2" in base["timed_on"]


def test_bench_gpus_mismatch_refused():
    """under a launcher, --gpus N must equal WORLD_SIZE (no silent 1-GPU run)"""
    env = _bench_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode == 2 and "WORLD_SIZE=2" in r.stderr


def test_bench_spawned_rank_failure_is_fatal():
    """a rank that fails makes `bench.py --gpus 2` exit non-zero with no line"""
    env = _bench_env(PAC_BENCH_MOCK_CONTEXT=os.path.join(ROOT, "tests", "no_such_mock.py"))
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1",
                        "--streams", "2", "--blocks-per-stream", "3"], capture_output=True, text=True, env=env,
                       timeout=300)
    assert r.returncode != 0 and r.stdout.strip() == ""


def test_bench_tail_lds_follows_the_kernel_source():
    """bench.py's occupancy limit of the dynamic-LDS tail comes from the
    kernel's own PAC_TAIL_LDS / PAC_TAIL_Q: 22 500 B, 4 waves"""
    b = _bench_module()
    assert b.dynamic_lds() == {"k_master_tail": (22500, 4)}
    assert b.csrc_defines(["PAC_NB", "WAVE"]) == {"PAC_NB": 25, "WAVE": 64}


def test_side_kernels_do_not_spill():
    """amdgpu_waves_per_eu(5) holds both k_master_lrms_spec instantiations
    (the <false> one: block switching, PAC_SIDE_CODED=0) without VGPR spills
    (ADVICE r05), per this build's resource report"""
    from pac_amd import build
    d = json.load(open(build.RESOURCES))
    if d.get("src_hash") != build.source_hash():
        pytest.skip("resource report of another build")
    for k in ("k_master_lrms_spec<true>", "k_master_lrms_spec<false>", "k_master_thr"):
        assert d["kernels"][k]["vgpr_spill"] == 0 and d["kernels"][k]["scratch_bytes_per_lane"] == 0, k
