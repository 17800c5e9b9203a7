"""pac_amd -- MI355X-native (gfx950) perceptual audio encoder.

Drop-in for the per-block encode path of wisamreid/Perceptual-Audio-Codec
(MDCT, psychoacoustic masking with M/S decision, bit-allocation water-fill,
block-floating-point quantizer, .pac/.wak bitstream) behind the reference's
own AudioFile / PCMFile / PACFile plugin surface.  The compute path is
hand-written HIP for CDNA4 in ``csrc/`` reached through the C-ABI
``include/pac_gpu.h`` (``libpacgpu.so``) via ctypes.

Modules mirror the reference's: ``audiofile``, ``pcmfile``, ``pacfile``,
``codec``, ``psychoac`` (band layout only), ``huffman``; plus ``synth``
(synthetic benchmark signals) and ``build`` (hipcc recipe).
"""
__version__ = "0.1.0"

PROFILE_ORIGIN = 0   # PerceptualAudioCodec_Origin/codec: .pac
PROFILE_MASTER = 1   # codec/: M/S + Huffman + bit reservoir, .wak
