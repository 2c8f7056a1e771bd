"""ccphylo_amd -- MI355X (gfx950) engine for ccphylo's `dist` and `tree` hot path.

Native pieces (built in-tree by ``__graft_entry__.build()`` / ``make -C ccphylo_amd``):
  lib/libccphylo_amd.so   HIP kernels + C-ABI (include/ccphylo_amd.h)
  lib/libccphylo_host.so  Phylip / Newick / FASTA host layer (include/ccphylo_host.h)
  bin/ccphylo             the `ccphylo dist` / `ccphylo tree` CLI

Python here is only a thin ctypes layer for tests and the benchmark.
"""
from .native import (CCG_TREE_DNJ, CCG_TREE_HNJ, CCG_TREE_NJ, CLI_PATH, CcgError, Device, ETYPES, JOIN_DTYPE,  # noqa: F401
                     engine_lib, host_lib, load_msa, load_phylip, newick_from_phylip)

__version__ = "0.1.0"
