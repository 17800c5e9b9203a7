"""AudioFile plugin protocol -- mirror of the reference's audiofile.py:51-92.

``CodingParams`` is the reference's attribute bag; ``AudioFile`` defines the
OpenForReading / OpenForWriting / ReadDataBlock / WriteDataBlock / Close
protocol that PCMFile and PACFile implement.
"""


class CodingParams:
    """A class to hold coding parameters to share across files (audiofile.py:51-53)."""
    pass


class AudioFile:
    """An abstract class defining handlers expected for a data file containing
    audio data (audiofile.py:56-92)."""

    def __init__(self, filename):
        self.filename = filename
        self.fp = None

    def OpenForReading(self):
        self.fp = open(self.filename, "rb")
        return self.ReadFileHeader()

    def OpenForWriting(self, codingParams):
        self.fp = open(self.filename, "wb")
        self.WriteFileHeader(codingParams)

    def Close(self, codingParams):
        self.fp.close()

    def ReadFileHeader(self):
        return CodingParams()

    def ReadDataBlock(self, codingParams):
        pass

    def WriteFileHeader(self, codingParams):
        pass

    def WriteDataBlock(self, data, codingParams):
        pass
