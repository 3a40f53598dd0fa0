"""Timing-only ablation source (wrong results, never shipped): the product
K_parse with single effects switchable off by -DMPC_ABL_* (exp/abl/abl.hip)."""
import os
R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
s = open(os.path.join(R, "minion-plasmid-consensus_amd/csrc/mpc_kernels.hip")).read()
subs = [
    ("      if (ok & (kind == 2) & !wrap & (TM != 3 || a.sub_wins == 0)) odd_sub(i, (int)pay);",
     "#ifndef MPC_ABL_NOSUB\n      if (ok & (kind == 2) & !wrap & (TM != 3 || a.sub_wins == 0)) odd_sub(i, (int)pay);\n#endif"),
    ("      if (del) {", "#ifdef MPC_ABL_NODEL\n      if (false) {\n#else\n      if (del) {\n#endif"),
    ("      if (ok & ((kind == 3) | wrap)) left_bit(gi);",
     "#ifndef MPC_ABL_NOLEFT\n      if (ok & ((kind == 3) | wrap)) left_bit(gi);\n#endif"),
    ("      if (TM == 3 && a.sub_wins > 0) {  // substitution events, wave-aggregated per window",
     "#ifdef MPC_ABL_NOSUB\n      if (false) {\n#else\n      if (TM == 3 && a.sub_wins > 0) {  // substitution events, wave-aggregated per window\n#endif"),
    ("      if (ballot(ins_inline))  // the event into its bucket's page (written once)",
     "#ifdef MPC_ABL_NOPLACE\n      if (false)\n#else\n      if (ballot(ins_inline))  // the event into its bucket's page (written once)\n#endif"),
    ("        if (ts < e2) { depth_inc(ts); depth_dec(e2); }",
     "#ifndef MPC_ABL_NOSPAN\n        if (ts < e2) { depth_inc(ts); depth_dec(e2); }\n#endif"),
]
subs += [
    ("          if (mine) wp[n0 + lanes_below(bw)] = (uint16_t)(((uint32_t)(i & (kSubWin - 1)) << 2) | pay);",
     "#ifndef MPC_ABL_NOSUBSTORE\n          if (mine) wp[n0 + lanes_below(bw)] = (uint16_t)(((uint32_t)(i & (kSubWin - 1)) << 2) | pay);\n#endif"),
    ("  if (fast) pg0[(old >> kPgBits) * kPgEv + (old & ((1u << kPgBits) - 1u))] = word;",
     "#ifndef MPC_ABL_NOEVSTORE\n  if (fast) pg0[(old >> kPgBits) * kPgEv + (old & ((1u << kPgBits) - 1u))] = word;\n#endif"),
]
for a, b in subs:
    assert s.count(a) == 1, a
    s = s.replace(a, b)
open(os.path.join(R, "exp/abl/abl.hip"), "w").write(s)
