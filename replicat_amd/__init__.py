"""replicat_amd -- an MI355X-native content-defined chunker for replicat.

The hot path (replicat's ``gclmulchunker``: keyed GF(2) hashes at 4-byte-aligned offsets,
cut at the windowed first argmax; /root/reference/src/adapters.cpp:42-77) runs as
hand-written gfx950 HIP kernels in ``libreplicat_chunker.so`` behind a C ABI
(``include/replicat_chunker.h``).  The Python side mirrors the reference's
``_replicat_adapters`` surface (``replicat_amd._replicat_adapters``) and adds a batch API over
many device- or host-resident streams (``replicat_amd.chunker``).
"""
__version__ = '0.3.0'
