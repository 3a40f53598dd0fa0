"""MI355X-native pileup + consensus: drop-in for the `consensus` rule of
scottdbrown/minion-plasmid-consensus (src/mapped_paf_read_parser.py).

Modules
  ingest   Steps 1-3 (FASTA / PAF ingest, flanks) -> packed per-read arrays
  engine   ctypes binding of libmpc.so (include/mpc.h) + torch device buffers
  writers  Step 7 output files
  synth    seeded synthetic cs-tagged data (tests / bench)
  dist     multi-GPU read sharding over RCCL (torch.distributed)
  mapped_paf_read_parser  the drop-in CLI
"""
from . import _build, ingest, writers, synth  # noqa: F401
from . import engine  # noqa: F401

__all__ = ["ingest", "engine", "writers", "synth"]
