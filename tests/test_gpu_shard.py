"""Multi-GPU sharding rehearsed on GPU 0: the file
batch of configs[3] split by pac_amd.shard.plan for virtual world sizes 1-4,
every rank's shard encoded by shard.encode_files in its own call, must give
exactly the bytes of the single-call encode (and of the reference's files
where the reference holds them).  No collective is involved: streams are
independent, so the shards only partition the work."""
import os

import pytest

from conftest import fixture

import pac_amd  # noqa: F401
from pac_amd import pacfile, shard

pytestmark = pytest.mark.gpu

NAMES = ["piano_test2", "percussion_test1", "speech_test3", "castanets", "daft", "piano_test1", "rock"]


@pytest.mark.parametrize("world", [1, 2, 3, 4])
def test_sharded_encode_equals_single_call(ctx, tmp_path, world):
    paths = [fixture(n + ".wav") for n in NAMES]
    single = [pacfile.encode_file(p, profile=pacfile.PROFILE_MASTER, context=ctx) for p in paths]
    outs = [str(tmp_path / ("%s.wak" % n)) for n in NAMES]
    done = []
    for rank in range(world):
        done += shard.encode_files(paths, outs, profile=pacfile.PROFILE_MASTER, context=ctx, rank=rank,
                                   world=world)
    assert sorted(done) == list(range(len(NAMES)))          # every stream exactly once
    for i, o in enumerate(outs):
        with open(o, "rb") as f:
            assert f.read() == single[i], NAMES[i]
    for n, b in zip(NAMES, single):                           # pinned where the reference holds the file
        if os.path.exists(fixture(n + ".wak")):
            with open(fixture(n + ".wak"), "rb") as f:
                assert b == f.read(), n
