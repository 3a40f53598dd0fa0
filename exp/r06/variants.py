#!/usr/bin/env python3
"""Round-6 experiment variants of libmpc.so: named text substitutions of the
product source (timing / counter variants; ablations give wrong results and are
never shipped).  Writes exp/v/src/<name>.hip (git-ignored) and builds
exp/v/<name>.so:   python3 exp/r06/variants.py name [name ...]   (or: all)"""
import os
import subprocess
import sys

R = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
SRC = os.path.join(R, "minion-plasmid-consensus_amd/csrc/mpc_kernels.hip")

S1_STORE = "        if (sev) a.subev[sev_base + nsub_s + lanes_below(bw)] = (uint16_t)(((uint32_t)i << 2) | pay);"
WIN_STORE = "          if (mine) wp[n0 + lanes_below(bw)] = (uint16_t)(((uint32_t)(i & (kSubWin - 1)) << 2) | pay);"
PG_STORE = "  if (fast) pg0[(old >> kPgBits) * kPgEv + (old & ((1u << kPgBits) - 1u))] = word;"
FAST = ("        fast = !v | (!lfar & ((olen >= 1) & (olen <= 4) & dig &\n"
        "                              (colon | minus | (star & (((bad >> shl) & 0xffu) == 0u)) | (plus & ((bad & vm) == 0u))) |\n"
        "                              nop));")

# (the lean / lazy / speculative / split variants of this round patched switches
# that commit b26663d holds and the product no longer does: build them from
# that commit's source)
VARIANTS = {
    "base": [],
    # counters: which store stream carries C5's write amplification
    "noevstore": [(PG_STORE, "")],
    "nosubstore": [(S1_STORE, ""), (WIN_STORE, "")],
    "subnt": [
        (S1_STORE, "        if (sev) __builtin_nontemporal_store((uint16_t)(((uint32_t)i << 2) | pay), "
                   "a.subev + sev_base + nsub_s + lanes_below(bw));"),
        (WIN_STORE, "          if (mine) __builtin_nontemporal_store((uint16_t)(((uint32_t)(i & (kSubWin - 1)) << 2) | pay), "
                    "wp + n0 + lanes_below(bw));"),
    ],
    # the per-unit check as VALU integers and one compare (fewer 64-bit mask ops);
    # a '*' needs all its operand bytes to be bases (not only the last)
    "intcheck_all": [("#define MPC_INT_CHECK_MODES 0x00", "#define MPC_INT_CHECK_MODES 0x1f")],
    "intcheck_old": [(FAST, """        {  // the check as VALU integers and one compare
          const uint32_t not4 = (uint32_t)(olen - 1) >> 2;  // 0 iff 1 <= olen <= 4
          const uint32_t dbad = (((Tx & 0x7F7F7F7Fu) + 0x76767676u) | Tx) & 0x80808080u & cvm;
          const uint32_t bbad = (star | plus) ? (bad & vm) : 0u;
          const uint32_t obad = (colon | star | plus | minus) ? 0u : 1u;
          fast = !v | (!lfar & (((not4 | dbad | bbad | obad) == 0u) | nop));
          (void)dig;
        }""")],
    # the next window's cs bytes loaded before the rounds
    "noflush": [("      if (dv) atomicAdd(a.diff + gb + p, dv);", "      (void)dv;"),
                ("      if (v) atomicAdd(sg + k, v);", "      (void)v; (void)sg;")],
    "defersub": [("#define MPC_DEFER_SUBEV 0", "#define MPC_DEFER_SUBEV 1")],
    "leftnosearch": [("      if (lb > la) {", "      if (lb < 0 && lb > la) {")],
    "leftnotally": [("          if (j < L) atomicAdd(tp + 4 * (L - 1 - j) + (int)((ev >> (2 * j)) & 3u), 1u);",
                     "          if (j < L && ev == 0x7fffffffu) atomicAdd(tp + 4 * (L - 1 - j) + (int)((ev >> (2 * j)) & 3u), 1u);")],
    "interp": [("#define MPC_LEFT_INTERP 0", "#define MPC_LEFT_INTERP 1")],
    "leftdiag": [("#ifdef MPC_LEFT_DIAG  // diagnostic builds only", "#define MPC_LEFT_DIAG\n#ifdef MPC_LEFT_DIAG  // diagnostic builds only")],
    "flushx2": [("#define MPC_FLUSH_X2 0", "#define MPC_FLUSH_X2 1")],
    "nodefer": [("#define MPC_DEFER_PLACE 1", "#define MPC_DEFER_PLACE 0")],
    "prefetch": [("#define MPC_PREFETCH_CS_MODES 0x00", "#define MPC_PREFETCH_CS_MODES 0x1f")],
    # both, in tally modes 1 and 2 only (short references: C1, C2)
    "m12opt": [("#define MPC_PREFETCH_CS_MODES 0x00", "#define MPC_PREFETCH_CS_MODES 0x06"),
               ("#define MPC_INT_CHECK_MODES 0x00", "#define MPC_INT_CHECK_MODES 0x06")],
    # timing upper bound of dropping the per-unit canonical check: no check, no
    # general decode (right results only on canonical input)
    "nocheck": [(FAST, "        fast = true; (void)dig; (void)bad; (void)vm; (void)nop; (void)lfar;"),
                ("        if (ballot(!fast)) return false;  // (before any effect: the round restarts on the general decode)",
                 "")],
}


def build(name):
    s = open(SRC).read()
    for a, b in VARIANTS[name]:
        assert s.count(a) == 1, (name, a[:80])
        s = s.replace(a, b)
    d = os.path.join(R, "exp/v/src")
    os.makedirs(d, exist_ok=True)
    src = os.path.join(d, name + ".hip")
    open(src, "w").write(s)
    out = os.path.join(R, "exp/v", name + ".so")
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-shared",
           "-I", os.path.join(R, "include"), "-I", os.path.join(R, "minion-plasmid-consensus_amd/csrc"), "-o", out, src]
    subprocess.run(cmd, check=True)
    print("built", out)


if __name__ == "__main__":
    names = list(VARIANTS) if sys.argv[1:] == ["all"] else sys.argv[1:]
    for n in names:
        build(n)
