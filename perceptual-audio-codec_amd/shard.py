"""Stream sharding across the GPUs of one node.

Streams (files) are independent: the only cross-block state is the 1-hop
overlap and, in the master profile, the per-stream bit reservoir.  Whole
streams are therefore assigned to ranks -- longest-processing-time first by
block count -- and each rank encodes its shard on its own GPU with one
``pac_encode_streams`` call.  There is no data-path collective; a barrier
ends the job.  (A single stream cannot be split in the master profile: its
reservoir chains every block to the next.)
"""
import os

import numpy as np


def blocks_of(n_frames, n_mdct_lines=1024):
    """Blocks the encoder emits for a stream of n_frames: every hop + the
    Close() flush block (pacfile.py:355-366)."""
    return (int(n_frames) + n_mdct_lines - 1) // n_mdct_lines + 1


def plan(block_counts, world):
    """LPT assignment: returns a list (per rank) of stream indices, each list in
    ascending stream order.  Deterministic (ties -> lower stream, lower rank)."""
    world = int(world)
    if world < 1:
        raise ValueError("world must be >= 1")
    order = sorted(range(len(block_counts)), key=lambda i: (-int(block_counts[i]), i))
    load = [0] * world
    shards = [[] for _ in range(world)]
    for i in order:
        r = min(range(world), key=lambda k: (load[k], k))
        shards[r].append(i)
        load[r] += int(block_counts[i])
    return [sorted(s) for s in shards]


def rank_env():
    return (int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")),
            int(os.environ.get("LOCAL_RANK", "0")))


def encode_files(in_paths, out_paths, profile=1, context=None, rank=None, world=None):
    """Encode this rank's shard of ``in_paths`` (all must share sample rate and
    channel count) into ``out_paths``; returns the indices it wrote."""
    from . import codec, pacfile
    from .pcmfile import read_for_encode
    r, w, local = rank_env()
    rank = r if rank is None else rank
    world = w if world is None else world
    reads = [read_for_encode(p) for p in in_paths]
    counts = [blocks_of(fr.shape[0]) for _, fr in reads]
    mine = plan(counts, world)[rank]
    if not mine:
        return []
    ctx = context or codec.default_context()
    fs = reads[mine[0]][0].sampleRate
    bodies = pacfile.encode_streams([reads[i][1] for i in mine], fs, profile, context=ctx)
    for i, body in zip(mine, bodies):
        cp = reads[i][0]
        with open(out_paths[i], "wb") as f:
            f.write(pacfile.header_bytes(cp.sampleRate, cp.nChannels, cp.numSamples) + body)
    return mine


def split_stream(n_frames, parts, n_mdct_lines=1024):
    """Split ONE stream's hops into up to `parts` contiguous ranges (SURVEY.md
    8(e), origin row: block ranges with a one-hop halo).  Returns a list of
    (frame_lo, frame_hi, flags): part i encodes hops [h_i, h_i+1) from frames
    [(h_i - 1) * 1024, h_i+1 * 1024) -- the first hop of that slice is the part's
    priorBlock (STREAM_HAS_PRIOR), every part but the last omits the Close()
    flush block (STREAM_NO_FLUSH).  The parts' data sections, concatenated in
    order, are the one-call data section.  Origin parts are independent (any
    rank, any order); master parts must run in order, each starting from the
    previous part's reservoir state."""
    from ._lib import STREAM_HAS_PRIOR, STREAM_NO_FLUSH
    n = int(n_frames)
    hops = (n + n_mdct_lines - 1) // n_mdct_lines
    parts = max(1, min(int(parts), hops))
    bounds = [hops * k // parts for k in range(parts + 1)]
    out = []
    for i in range(parts):
        h0, h1 = bounds[i], bounds[i + 1]
        lo = (h0 - 1) * n_mdct_lines if i > 0 else 0
        hi = min(n, h1 * n_mdct_lines)
        flags = (STREAM_HAS_PRIOR if i > 0 else 0) | (STREAM_NO_FLUSH if i < parts - 1 else 0)
        out.append((lo, hi, flags))
    return out


def balance(block_counts, shards):
    loads = np.array([sum(int(block_counts[i]) for i in s) for s in shards], dtype=np.int64)
    return loads, (loads.max() / max(loads.mean(), 1e-9)) if len(loads) else 1.0
