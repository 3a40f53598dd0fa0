"""MI355X-native pileup + consensus (drop-in for src/mapped_paf_read_parser.py)."""
