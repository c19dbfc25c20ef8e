"""oxen_amd -- MI355X-native content-hashing stage for Oxen's `oxen add` / commit indexing path.

XXH3-128 (the digest liboxen stores for every file, util/hasher.rs) computed by hand-written
gfx950 HIP kernels behind the C ABI in include/oxen_hash.h (oxen_amd/liboxen_hash.so).

Modules:
  hasher    -- mirror of liboxen `util::hasher` (same names / errors) plus batched forms
  merkle    -- MerkleHash and the commit-time parent-node streams (K2)
  version_store -- verify-before-publish writes (AtomicFile.with_hash, LocalVersionStore)
  dedup     -- fixed-size and FastCDC chunking + chunk digests (block-level dedup)
  procpool  -- file hashing sharded over reader processes (the open/close floor is per process)
  shard     -- multi-GPU sharding and the RCCL digest gather
  device    -- device-resident (HBM) batch entry points over torch buffers
  workloads -- deterministic synthetic inputs for the BASELINE.json configs
  build     -- hipcc build of the in-tree library
"""
from ._capi import OxenError  # noqa: F401

__version__ = "0.1.0"
