"""objectkv_amd -- MI355X-native SST block encode/decode for ObjectKV's
segment format (drop-in under danthegoodman1/ObjectKV's sst package).

The hot path is libokv_sst.so (HIP kernels for gfx950 behind the C-ABI in
include/okv_sst.h).  Importing this package does not touch the GPU.
"""
from ._lib import build, lib  # noqa: F401
from .sst import (Decoded, Decoder, Encoded, Encoder, GpuSegmentWriter, Metadata,  # noqa: F401
                  OkvError, SegmentWriter, bytes_to_metadata, fetch_metadata, pack_rows,
                  synth_segment, xxh64)

__all__ = ["build", "lib", "Decoder", "Decoded", "Encoder", "Encoded", "GpuSegmentWriter",
           "Metadata", "OkvError", "SegmentWriter", "pack_rows",
           "bytes_to_metadata", "fetch_metadata", "synth_segment", "xxh64"]
