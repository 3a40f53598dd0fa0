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

VARIANTS = {
    "base": [],
    # (round 6: "nosplit" -- one loop, a non-canonical round retried in place --
    # became the default; "split" is the two-loop dispatch)
    "split": [("#define MPC_SPLIT_ROUNDS 0", "#define MPC_SPLIT_ROUNDS 1")],
    # speculative pass without the long-operand decode (long ':' / '+' fail over)
    "spnolong": [("          if (ballot(lng & (colon | plus))) {  // rare: the long operand bytewise from the stage",
                  "          xok = false;\n          if (false) {")],
    # the exact K_parse alone (no speculative pass)
    "nospec": [("#define MPC_SPEC_PARSE 1", "#define MPC_SPEC_PARSE 0")],
    # windows checked once (byte masks), their rounds without the per-unit check
    "lean": [("#define MPC_LEAN_WINDOWS 0", "#define MPC_LEAN_WINDOWS 1")],
    # ... the other windows on the general decode only (two loops, not three)
    "lean2": [("#define MPC_LEAN_WINDOWS 0", "#define MPC_LEAN_WINDOWS 2")],
    # structure checked per window, characters per round
    "lean3": [("#define MPC_LEAN_WINDOWS 0", "#define MPC_LEAN_WINDOWS 3")],
    # timing: the per-unit check computed, no branch on it (a speculation flag
    # ORed per lane; right results only on canonical input)
    "nobranch": [("    const int far_c = (int)(C - A < (1 << 30) ? C - A : (1 << 30));  // wave-uniform",
                  "    const int far_c = (int)(C - A < (1 << 30) ? C - A : (1 << 30));  // wave-uniform\n    uint32_t spec_bad = 0;"),
                 ("          if (ballot(!fast)) return false;  // (before any effect: the round restarts on the general decode)",
                  "          spec_bad |= fast ? 0u : 1u;"),
                 ("    // ---- reads that ended in this window: i_end; carry the open one ----",
                  "    if (ballot(spec_bad != 0u) && l == 0) atomicOr(&a.status[7], 1u);\n"
                  "    // ---- reads that ended in this window: i_end; carry the open one ----")],
    # diagnostics: windows counted in status[6] (all) / status[7] (not lean)
    "leandiag": [("#define MPC_LEAN_WINDOWS 0", "#define MPC_LEAN_WINDOWS 2"),
                 ("        lean = !far && !ballot(bad != 0);",
                  "        lean = !far && !ballot(bad != 0);\n"
                  "        if (l == 0) { atomicAdd(&a.status[6], 1u); if (!lean) atomicAdd(&a.status[7], 1u); }")],
    # timing: every window lean (no check; right results only on canonical input)
    "leanforce": [("#define MPC_LEAN_WINDOWS 0", "#define MPC_LEAN_WINDOWS 2"),
                  ("        lean = !far && !ballot(bad != 0);", "        lean = !far; (void)bad;")],
    # no slot reads in the common round (read index from the slot number)
    "lazy": [("#define MPC_SLOT_LAZY 0", "#define MPC_SLOT_LAZY 1")],
    "lean2lazy": [("#define MPC_LEAN_WINDOWS 0", "#define MPC_LEAN_WINDOWS 2"),
                  ("#define MPC_SLOT_LAZY 0", "#define MPC_SLOT_LAZY 1")],
    # counters: which store stream carries C5's write amplification
    "noevstore": [(PG_STORE, "")],
    "nosubstore": [(S1_STORE, ""), (WIN_STORE, "")],
    "subnt": [
        (S1_STORE, "        if (sev) __builtin_nontemporal_store((uint16_t)(((uint32_t)i << 2) | pay), "
                   "a.subev + sev_base + nsub_s + lanes_below(bw));"),
        (WIN_STORE, "          if (mine) __builtin_nontemporal_store((uint16_t)(((uint32_t)(i & (kSubWin - 1)) << 2) | pay), "
                    "wp + n0 + lanes_below(bw));"),
    ],
    # timing upper bound of a window-level canonical check: the per-round
    # validity predicate and the general-decode branch dropped (right results
    # only on canonical input, which the synthetic configs are)
    "nocheck": [(FAST, "        fast = true; (void)dig; (void)bad; (void)vm; (void)nop; (void)lfar;"),
                ("      if (!fast_decode<TM>() || ballot(!fast)) {  // general decode of the whole round",
                 "      if (!fast_decode<TM>()) {  // general decode of the whole round")],
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
