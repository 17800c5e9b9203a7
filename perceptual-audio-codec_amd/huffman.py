"""Huffman coder state -- mirror of the reference's ``Huffman`` class
(Huffman.py:253-374) for the plugin surface.

The 10 static tables are read from ``data/huffman_tables.bin`` (a neutral
export of the reference's huffmanTables.pickle made without unpickling, see
tests/golden/export_huffman_tables.py) and uploaded to the GPU by
``_lib.Context``.  Table selection, code emission and the reservoir updates of
the encode path run in the HIP kernels (k_master_tail / k_master_pack); this
class carries the reference's mutable ``bitDeposit`` between per-block calls
and exposes the reference's reservoir methods with the same semantics.
"""
import os
import struct

HERE = os.path.dirname(os.path.abspath(__file__))
TABLES = os.path.join(HERE, "data", "huffman_tables.bin")


def load_tables(path=TABLES):
    """{tableID: {symbol: code string, -1: escape code string}} (Huffman.py:149-153)."""
    with open(path, "rb") as f:
        d = f.read()
    if d[:8] != b"PACHUF01":
        raise ValueError("not a PACHUF01 table image")
    n = struct.unpack_from("<I", d, 8)[0]
    o = 12
    tables = {}
    for _ in range(n):
        tid, ne, el, eb = struct.unpack_from("<IIII", d, o)
        o += 16
        enc = {-1: format(eb, "0%db" % el)}
        for _ in range(ne):
            s, ln, b = struct.unpack_from("<iII", d, o)
            o += 12
            enc[s] = format(b, "0%db" % ln)
        tables[tid] = enc
    return tables


class Huffman:
    """Reservoir + tables of the WAK coder (Huffman.py:253-374)."""

    ESCAPE_CODE = -1

    def __init__(self, path=TABLES):
        self.huffmanTables = load_tables(path)
        self.bitDeposit = 0

    def depositBits(self, numBits):          # Huffman.py:353-354
        self.bitDeposit += numBits

    def withdrawBits(self):                  # Huffman.py:363-371 (Py2 floor division)
        extraBit = 0
        if self.bitDeposit > 10:
            extraBit = self.bitDeposit // 100
            self.bitDeposit -= extraBit
        elif self.bitDeposit < 0:
            extraBit = self.bitDeposit
            self.bitDeposit = 0
        return extraBit

    def getBitDeposit(self):
        return self.bitDeposit
