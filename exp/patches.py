PATCHES = {
  # skip the rounds (window overhead + epilogue only)
  "norounds": [("    for (int t0 = 0; t0 < T; t0 += 64) {", "    for (int t0 = 0; t0 < T && T < 0; t0 += 64) {")],
  # skip the epilogue
  "noepi": [("  parse_epilogue<TM>(a, n, gb, nbk, r0, hl, bcnt, uni, wcnt, wbase, nw, reinterpret_cast<uint64_t*>(lds),\n                     nw * (int)sizeof(WL) / 8);",
             "  if (a.n_reads < 0) parse_epilogue<TM>(a, n, gb, nbk, r0, hl, bcnt, uni, wcnt, wbase, nw, reinterpret_cast<uint64_t*>(lds),\n                     nw * (int)sizeof(WL) / 8);")],
}
PATCHES["ld4"] = [(
"""      const uint32_t* b32 = reinterpret_cast<const uint32_t*>(W.stage);
      const int a4 = sx >> 2;
      const uint32_t sh = (uint32_t)(sx & 3);
      const uint32_t d0 = b32[a4], d1 = b32[a4 + 1], d2 = b32[a4 + 2];
      const uint32_t x0 = __builtin_amdgcn_alignbyte(d1, d0, sh);
      const uint32_t x1 = __builtin_amdgcn_alignbyte(d2, d1, sh);""",
"""      const uint32_t* b32 = reinterpret_cast<const uint32_t*>(W.stage);
      const int b4 = s0 >> 2;  // the unit's 16 bytes from its start's dword: ':' operand, op, 4 operand bytes
      const uint32_t D0 = b32[b4], D1 = b32[b4 + 1], D2 = b32[b4 + 2], D3 = b32[b4 + 3];
      const int offx = sx - 4 * b4;  // 0..8
      const uint32_t sh = (uint32_t)(offx & 3);
      const int kx = offx >> 2;
      const uint32_t lo_ = kx == 0 ? D0 : (kx == 1 ? D1 : D2);
      const uint32_t mi_ = kx == 0 ? D1 : (kx == 1 ? D2 : D3);
      const uint32_t hi_ = kx == 0 ? D2 : D3;
      const uint32_t x0 = __builtin_amdgcn_alignbyte(mi_, lo_, sh);
      const uint32_t x1 = __builtin_amdgcn_alignbyte(hi_, mi_, sh);"""),
("""      const int pa = (s0 + 1) >> 2;
      const uint32_t pw = __builtin_amdgcn_alignbyte(b32[pa + 1], b32[pa], (uint32_t)((s0 + 1) & 3));""",
"""      const int offp = s0 + 1 - 4 * b4;  // 1..4
      const bool kp = offp >= 4;
      const uint32_t pw = __builtin_amdgcn_alignbyte(kp ? D2 : D1, kp ? D1 : D0, (uint32_t)(offp & 3));""")]
PATCHES["sel"] = [(
"""      uint32_t pay = star ? ((codes >> shl) & 3u) : (pk & ((1u << (2 * ol4)) - 1u));""",
"""      const uint32_t mstar = 0u - (uint32_t)star;
      uint32_t pay = (mstar & ((codes >> shl) & 3u)) | (~mstar & (pk & ((1u << (2 * ol4)) - 1u)));"""),
("""      int kind = !act ? 0 : colon ? (adv_c > 0 ? 1 : 0) : (olen <= 0) ? 0 : star ? 2 : plus ? 3 : minus ? 4 : 0;
      int adv = kind == 1 ? adv_c : kind == 2 ? 1 : kind == 4 ? (olen < kAdvCap ? olen : kAdvCap) : 0;""",
"""      const int kop = ((int)star << 1) | ((int)plus * 3) | ((int)minus << 2);  // exclusive classes
      const int mcol = -(int)colon;
      int kind = (-(int)act) & ((mcol & (int)(adv_c > 0)) | (~mcol & (-(int)(olen > 0) & kop)));
      int adv = (-(int)(kind == 1) & adv_c) | (int)(kind == 2) | (-(int)(kind == 4) & (olen < kAdvCap ? olen : kAdvCap));""")]
PATCHES["tokpf"] = [(
"""    for (int t0 = 0; t0 < T; t0 += 64) {
      const int t = t0 + l;
      const bool v = t < T;
      const uint32_t t0r = W.tok[t], t1r = W.tok[t + 1];  // in bounds for every lane (+64 padding)""",
"""    constexpr int kTokLast = tok_cap<WIN>() + 2 + 64 - 2;
    uint32_t nt0 = W.tok[l], nt1 = W.tok[l + 1];
    for (int t0 = 0; t0 < T; t0 += 64) {
      const int t = t0 + l;
      const bool v = t < T;
      const uint32_t t0r = nt0, t1r = nt1;  // in bounds for every lane (+64 padding)
      {  // the next round's entries, loaded before this round's LDS traffic
        const int tn = min(t + 64, kTokLast);
        nt0 = W.tok[tn]; nt1 = W.tok[tn + 1];
      }""")]
PATCHES["late"] = [(
"""      //   bases: (c|0x20) must equal "acgt"[h] with h = (lc>>1)&3 (v_perm table lookup)
      const uint32_t lc = w0 | 0x20202020u;
      const uint32_t hh = (lc >> 1) & 0x03030303u;
      const uint32_t bad = lc ^ __builtin_amdgcn_perm(0u, 0x67746361u, hh);
      const uint32_t codes = ((hh & 0x01010101u) << 1) | ((hh >> 1) & 0x01010101u);  // dict order A0 T1 C2 G3
      const int shl = 8 * ((olen - 1) & 3);
      const bool last_ok = ((bad >> shl) & 0xffu) == 0;  // '*': written base = operand[-1] (:96)
      uint32_t pk = codes;
      pk = (pk | (pk >> 6)) & 0x000f000fu;
      pk = (pk | (pk >> 12)) & 0xffu;
      uint32_t pay = star ? ((codes >> shl) & 3u) : (pk & ((1u << (2 * ol4)) - 1u));
      const bool slow = lfar | (pre & !cdig) | (act & ((colon & !dig_ok) | ((star | plus) & (olen > 4))));
      int kind = !act ? 0 : colon ? (adv_c > 0 ? 1 : 0) : (olen <= 0) ? 0 : star ? 2 : plus ? 3 : minus ? 4 : 0;
      int adv = kind == 1 ? adv_c : kind == 2 ? 1 : kind == 4 ? (olen < kAdvCap ? olen : kAdvCap) : 0;
      uint32_t err = (v & !spec) ? DE_OP : 0u;  // cs does not start with an operator (:100-102)
      if (act & star & (olen == 0)) err |= DE_INDEX;  // operand[-1] of '' (:96)
      if ((kind == 2) & !last_ok) err |= DE_KEY;
      if ((kind == 3) & ((bad & vm) != 0)) err |= DE_KEY;
      int olen_e = olen;
      if (slow) {  // rare: decode from HBM
        const int64_t s = A + sx, e = A + ex64;
        const TokInfo ti = analyze_long(a.cs, s, e, last);
        adv = ti.adv; kind = ti.kind; pay = ti.pay; err = ti.err;
        olen_e = (int)(e - s - 1 < kAdvCap ? e - s - 1 : kAdvCap);
        if (pl) {
          const TokInfo tp = analyze_long(a.cs, A + s0, s, false);
          adv0 = tp.adv;
          err |= tp.err;
        }
      }""",
"""      const bool slow = lfar | (pre & !cdig) | (act & ((colon & !dig_ok) | ((star | plus) & (olen > 4))));
      const int kop = ((int)star << 1) | ((int)plus * 3) | ((int)minus << 2);  // exclusive classes
      const int mcol = -(int)colon;
      int kind = (-(int)act) & ((mcol & (int)(adv_c > 0)) | (~mcol & (-(int)(olen > 0) & kop)));
      int adv = (-(int)(kind == 1) & adv_c) | (int)(kind == 2) | (-(int)(kind == 4) & (olen < kAdvCap ? olen : kAdvCap));
      int olen_e = olen;
      uint32_t s_pay = 0u, s_err = 0u;
      if (slow) {  // rare: decode from HBM
        const int64_t s = A + sx, e = A + ex64;
        const TokInfo ti = analyze_long(a.cs, s, e, last);
        adv = ti.adv; kind = ti.kind; s_pay = ti.pay; s_err = ti.err;
        olen_e = (int)(e - s - 1 < kAdvCap ? e - s - 1 : kAdvCap);
        if (pl) {
          const TokInfo tp = analyze_long(a.cs, A + s0, s, false);
          adv0 = tp.adv;
          s_err |= tp.err;
        }
      }"""),
("""      const int i = iu + adv0;                // ... and at its main token
""",
"""      const int i = iu + adv0;                // ... and at its main token
      // payload and data errors of the fast decode (after the scans: they do not feed the coordinates)
      uint32_t pay, err;
      {
        //   bases: (c|0x20) must equal "acgt"[h] with h = (lc>>1)&3 (v_perm table lookup)
        const uint32_t lc = w0 | 0x20202020u;
        const uint32_t hh = (lc >> 1) & 0x03030303u;
        const uint32_t bad = lc ^ __builtin_amdgcn_perm(0u, 0x67746361u, hh);
        const uint32_t codes = ((hh & 0x01010101u) << 1) | ((hh >> 1) & 0x01010101u);  // dict order A0 T1 C2 G3
        const int shl = 8 * ((olen - 1) & 3);
        const bool last_ok = ((bad >> shl) & 0xffu) == 0;  // '*': written base = operand[-1] (:96)
        uint32_t pk = codes;
        pk = (pk | (pk >> 6)) & 0x000f000fu;
        pk = (pk | (pk >> 12)) & 0xffu;
        const uint32_t mstar = 0u - (uint32_t)star;
        const uint32_t f_pay = (mstar & ((codes >> shl) & 3u)) | (~mstar & (pk & ((1u << (2 * ol4)) - 1u)));
        uint32_t f_err = (v & !spec) ? DE_OP : 0u;  // cs does not start with an operator (:100-102)
        if (act & star & (olen == 0)) f_err |= DE_INDEX;  // operand[-1] of '' (:96)
        if ((kind == 2) & !last_ok) f_err |= DE_KEY;
        if ((kind == 3) & ((bad & vm) != 0)) f_err |= DE_KEY;
        pay = slow ? s_pay : f_pay;
        err = slow ? s_err : f_err;
      }
""")]
PATCHES["dppnx"] = [(
"""    const int64_t o_nx = __shfl(cur.o, (l + 1) & 63, 64);
    const uint32_t uo_nx = (uint32_t)__shfl((int)cur.uo, (l + 1) & 63, 64);
    const uint32_t dno_nx = (uint32_t)__shfl((int)cur.dno, (l + 1) & 63, 64);""",
"""    // lane l < 63: read rs0 + l + 1's offsets (DPP wave shift, no LDS permute)
    const int64_t o_nx = (int64_t)(((uint64_t)from_lane_above((uint32_t)((uint64_t)cur.o >> 32)) << 32) |
                                   from_lane_above((uint32_t)cur.o));
    const uint32_t uo_nx = from_lane_above(cur.uo);
    const uint32_t dno_nx = from_lane_above(cur.dno);""")]
PATCHES["flank4"] = [(
"""      for (int x = tid; x < cn; x += blockDim.x) {
        const uint32_t word = bm[x >> 5];
        const int o = wpre[x >> 5] + __popc(word & (0xffffffffu >> (31 - (x & 31))));  // owner: starts <= x
        const int32_t rw = t_row[o];
        if (rw < 0) continue;
        const int64_t row = (int64_t)rw + (c0 + x - t_start[o]);
        const int code = code_exact(stage[x + sh0]);
        if (code < 0) { lerr |= DE_KEY; const int64_t rr = r0 + t_read[o]; lread = rr < lread ? rr : lread; continue; }
        const int64_t wr = row - w0;
        if (wr >= 0 && wr < kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
        else atomicAdd(a.rows + row * 4 + code, 1u);
      }""",
"""      // 4 bytes per thread per step (strided by the block: consecutive lanes
      // stay on consecutive bytes), their LDS reads batched
      constexpr int kFU = 4;
      for (int xb = tid; xb < cn; xb += kFU * kFR) {
        int o[kFU], x[kFU];
#pragma unroll
        for (int u = 0; u < kFU; ++u) {
          x[u] = xb + u * kFR;
          const int xc = x[u] < cn ? x[u] : (int)cn - 1;
          const uint32_t word = bm[xc >> 5];
          o[u] = wpre[xc >> 5] + __popc(word & (0xffffffffu >> (31 - (xc & 31))));  // owner: starts <= x
        }
        int32_t rw[kFU], st[kFU];
        uint32_t by[kFU];
#pragma unroll
        for (int u = 0; u < kFU; ++u) {
          rw[u] = t_row[o[u]];
          st[u] = t_start[o[u]];
          by[u] = stage[(x[u] < cn ? x[u] : (int)cn - 1) + sh0];
        }
#pragma unroll
        for (int u = 0; u < kFU; ++u) {
          if (x[u] >= cn || rw[u] < 0) continue;
          const int64_t row = (int64_t)rw[u] + (c0 + x[u] - st[u]);
          const int code = code_exact(by[u]);
          if (code < 0) { lerr |= DE_KEY; const int64_t rr = r0 + t_read[o[u]]; lread = rr < lread ? rr : lread; continue; }
          const int64_t wr = row - w0;
          if (wr >= 0 && wr < kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
          else atomicAdd(a.rows + row * 4 + code, 1u);
        }
      }""")]
PATCHES["fl_noflush"] = [("""      if (v) atomicAdd(a.rows + w0 * 4 + k, v);
    }
  }
  if (lerr) {""", """      if (v && a.N < 0) atomicAdd(a.rows + w0 * 4 + k, v);
    }
  }
  if (lerr) {""")]
PATCHES["fl_noatom"] = [("""        if (wr >= 0 && wr < kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
        else atomicAdd(a.rows + row * 4 + code, 1u);
      }""", """        if (wr >= 0 && wr < kWinRows) { if (a.N < 0) atomicAdd(wn + wr * 5 + code, 1u); }
        else if (a.N < 0) atomicAdd(a.rows + row * 4 + code, 1u);
      }""")]
PATCHES["fl_noglob"] = [("""        if (wr >= 0 && wr < kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
        else atomicAdd(a.rows + row * 4 + code, 1u);
      }""", """        if (wr >= 0 && wr < kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
        else if (a.N < 0) atomicAdd(a.rows + row * 4 + code, 1u);
      }""")]
PATCHES["fl_noloop"] = [("""      for (int x = tid; x < cn; x += blockDim.x) {
        const uint32_t word = bm[x >> 5];""", """      for (int x = tid; x < cn && a.N < 0; x += blockDim.x) {
        const uint32_t word = bm[x >> 5];""")]
PATCHES["clr16"] = [("""    const uint32_t v = c.value[k];
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < c.words[k]; i += stride) p[i] = v;
  }""", """    const uint32_t v = c.value[k];
    const int64_t nw = c.words[k], t0 = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // 16-byte stores between a 4-byte head (to 16-byte alignment) and tail
    int64_t head = (int64_t)(((16u - ((uint32_t)(uintptr_t)p & 15u)) & 15u) >> 2);
    head = head < nw ? head : nw;
    if (t0 < head) p[t0] = v;
    const int64_t nq = (nw - head) >> 2;
    uint4* q = reinterpret_cast<uint4*>(p + head);
    const uint4 vv = make_uint4(v, v, v, v);
    for (int64_t i = t0; i < nq; i += stride) q[i] = vv;
    const int64_t t1 = head + 4 * nq;
    if (t0 < nw - t1) p[t1 + t0] = v;
  }""")]
PATCHES["fl_count"] = [("""        if (wr >= 0 && wr < kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
        else atomicAdd(a.rows + row * 4 + code, 1u);
      }""", """        const bool hit = wr >= 0 && wr < kWinRows;
        if (hit) atomicAdd(wn + wr * 5 + code, 1u);
        else atomicAdd(a.rows + row * 4 + code, 1u);
        { const uint64_t bh = ballot(hit), bm_ = ballot(!hit);
          if (lane() == __ffsll((unsigned long long)(bh | bm_)) - 1) {
            atomicAdd(&a.status[5], (uint32_t)__popcll(bh)); atomicAdd(&a.status[6], (uint32_t)__popcll(bm_)); atomicAdd(&a.status[7], 1u); } }
      }""")]
PATCHES["p_notally"] = [("""        if (kind == 2 && (TM != 3 || a.sub_wins == 0)) odd_sub(i, (int)pay);
        if (kind == 4 && i >= 0 && i < n) {""", """        if (kind == 2 && (TM != 3 || a.sub_wins == 0) && a.n_reads < 0) odd_sub(i, (int)pay);
        if (kind == 4 && i >= 0 && i < n && a.n_reads < 0) {""")]
PATCHES["p_noins"] = [("""      if (ins_inline) {
        a.ins_raw[ev_base + nev + lanes_below(bins)] = ins_event(i, olen_e, pay, a.read_offset + rl);
        atomicAdd(bcnt + i / kBW, 1u);
      }""", """      if (ins_inline && a.n_reads < 0) {
        a.ins_raw[ev_base + nev + lanes_below(bins)] = ins_event(i, olen_e, pay, a.read_offset + rl);
        atomicAdd(bcnt + i / kBW, 1u);
      }""")]
PATCHES["p_noscan"] = [("const int ainc = wave_scan_i32(advu);", "const int ainc = advu * (l + 1);"),
                       ("const int aex_rs = wave_scan_max_i32(is_rs ? aex : 0);", "const int aex_rs = is_rs ? aex : 0;")]
PATCHES["p_nomax"] = [("const int aex_rs = wave_scan_max_i32(is_rs ? aex : 0);", "const int aex_rs = is_rs ? aex : 0;")]
PATCHES['two'] = [('    // ---- rounds: one token per lane ----\n    int32_t G = 0;  // advances of the window\'s earlier rounds\n    int qc = 0;     // read starts of the window\'s earlier rounds\n    for (int t0 = 0; t0 < T; t0 += 64) {\n      const int t = t0 + l;\n      const bool v = t < T;\n      const uint32_t t0r = W.tok[t], t1r = W.tok[t + 1];  // in bounds for every lane (+64 padding)\n      const uint32_t e0 = v ? t0r : 0u, e1 = v ? t1r : 0u;\n      const int s0 = (int)(e0 & 0xfffu);         // unit start\n      const int pl = (int)((e0 >> 12) & 7u);     // \':\' operand length of a unit\'s prefix (0: none)\n      const int sx = pl ? s0 + pl + 1 : s0;      // the unit\'s main token\n      const bool lfar = v && ((e1 & 0x7fffu) == kFar);\n      const int64_t ex64 = lfar ? C - A : (int64_t)(e1 & 0xfffu);  // far: the token ends at C (beyond the window)\n      const int ex = (int)(ex64 - sx - 1 < kAdvCap ? ex64 : sx + 1 + kAdvCap);\n      const bool is_rs = v && (e0 >> 15);\n      const bool last = v && (e1 >> 15);\n      const uint64_t brs = ballot(is_rs);\n      const int q = qc + lanes_below(brs) + (is_rs ? 1 : 0);\n      // the read\'s slot, loaded before the decode (a read starting in this\n      // round needs no s_val: see the coordinates below)\n      const int32_t q_val = W.s_val[q], q_ts = W.s_ts[q], q_read = W.s_read[q], q_iend = W.s_iend[q];\n      // fast decode from the staged bytes: op, then 4 operand bytes\n      const uint32_t* b32 = reinterpret_cast<const uint32_t*>(W.stage);\n      const int a4 = sx >> 2;\n      const uint32_t sh = (uint32_t)(sx & 3);\n      const uint32_t d0 = b32[a4], d1 = b32[a4 + 1], d2 = b32[a4 + 2];\n      const uint32_t x0 = __builtin_amdgcn_alignbyte(d1, d0, sh);\n      const uint32_t x1 = __builtin_amdgcn_alignbyte(d2, d1, sh);\n      const uint32_t op = x0 & 0xffu;\n      const uint32_t w0 = __builtin_amdgcn_alignbyte(x1, x0, 1u);\n      const int olen = ex - sx - 1;\n      // branch-free decode: op class, 4 operand bytes at once (SWAR)\n      const bool colon = op == \':\', star = op == \'*\', plus = op == \'+\', minus = op == \'-\';\n      const bool spec = colon | star | plus | minus | (op == \'Z\');\n      const bool act = v & spec & ((olen > 0) | last);  // empty operand: skipped unless last (:309, :320)\n      const int ol4 = olen < 0 ? 0 : (olen > 4 ? 4 : olen);\n      const uint32_t vm = ol4 == 4 ? 0xffffffffu : ((1u << (8 * ol4)) - 1u);  // operand bytes in w0\n      //   the unit\'s \':\' operand -- its prefix (pl bytes after s0) or the main\n      //   token\'s own operand -- up to 4 digits: right-align, SWAR decimal\n      const bool pre = pl != 0;\n      const int pa = (s0 + 1) >> 2;\n      const uint32_t pw = __builtin_amdgcn_alignbyte(b32[pa + 1], b32[pa], (uint32_t)((s0 + 1) & 3));\n      const int cl = pre ? pl : (colon ? ol4 : 0);\n      const uint32_t cw = pre ? pw : w0;\n      const uint32_t cvm = cl == 4 ? 0xffffffffu : ((1u << (8 * cl)) - 1u);\n      const uint32_t Tx = cw ^ 0x30303030u;\n      const bool cdig = ((((Tx & 0x7F7F7F7Fu) + 0x76767676u) | Tx) & 0x80808080u & cvm) == 0;\n      uint32_t X = cl == 0 ? 0u : (Tx & cvm & 0x0F0F0F0Fu) << (8 * (4 - cl));\n      X = mul2561(X) >> 8;\n      X = ((X & 0x00FF00FFu) * 6553601u) >> 16;\n      const int adv_c = (int)(X & 0xffffu);\n      int adv0 = pre ? adv_c : 0;\n      const bool dig_ok = (olen >= 1) & (olen <= 4) & cdig;  // main \':\' token\n      //   bases: (c|0x20) must equal "acgt"[h] with h = (lc>>1)&3 (v_perm table lookup)\n      const uint32_t lc = w0 | 0x20202020u;\n      const uint32_t hh = (lc >> 1) & 0x03030303u;\n      const uint32_t bad = lc ^ __builtin_amdgcn_perm(0u, 0x67746361u, hh);\n      const uint32_t codes = ((hh & 0x01010101u) << 1) | ((hh >> 1) & 0x01010101u);  // dict order A0 T1 C2 G3\n      const int shl = 8 * ((olen - 1) & 3);\n      const bool last_ok = ((bad >> shl) & 0xffu) == 0;  // \'*\': written base = operand[-1] (:96)\n      uint32_t pk = codes;\n      pk = (pk | (pk >> 6)) & 0x000f000fu;\n      pk = (pk | (pk >> 12)) & 0xffu;\n      const uint32_t mstar = 0u - (uint32_t)star;\n      uint32_t pay = (mstar & ((codes >> shl) & 3u)) | (~mstar & (pk & ((1u << (2 * ol4)) - 1u)));\n      const bool slow = lfar | (pre & !cdig) | (act & ((colon & !dig_ok) | ((star | plus) & (olen > 4))));\n      const int kop = ((int)star << 1) | ((int)plus * 3) | ((int)minus << 2);  // exclusive classes\n      const int mcol = -(int)colon;\n      int kind = (-(int)act) & ((mcol & (int)(adv_c > 0)) | (~mcol & (-(int)(olen > 0) & kop)));\n      int adv = (-(int)(kind == 1) & adv_c) | (int)(kind == 2) | (-(int)(kind == 4) & (olen < kAdvCap ? olen : kAdvCap));\n      uint32_t err = (v & !spec) ? DE_OP : 0u;  // cs does not start with an operator (:100-102)\n      if (act & star & (olen == 0)) err |= DE_INDEX;  // operand[-1] of \'\' (:96)\n      if ((kind == 2) & !last_ok) err |= DE_KEY;\n      if ((kind == 3) & ((bad & vm) != 0)) err |= DE_KEY;\n      int olen_e = olen;\n      if (slow) {  // rare: decode from HBM\n        const int64_t s = A + sx, e = A + ex64;\n        const TokInfo ti = analyze_long(a.cs, s, e, last);\n        adv = ti.adv; kind = ti.kind; pay = ti.pay; err = ti.err;\n        olen_e = (int)(e - s - 1 < kAdvCap ? e - s - 1 : kAdvCap);\n        if (pl) {\n          const TokInfo tp = analyze_long(a.cs, A + s0, s, false);\n          adv0 = tp.adv;\n          err |= tp.err;\n        }\n      }\n      // ---- coordinates ----\n      const int advu = adv0 + adv;            // unit advance <= 2^21: 64 lanes stay < 2^31\n      const int ainc = wave_scan_i32(advu);\n      const int aex = ainc - advu;\n      const int atot = wave_last_i32(ainc);\n      // a read starting in this round (rs lane j <= l): i = tstart + the\n      // advances since lane j = aex - aex(j); aex never decreases, so aex(j)\n      // is a max-scan over the rs lanes (DPP: no LDS round trip)\n      const int aex_rs = wave_scan_max_i32(is_rs ? aex : 0);\n      if (is_rs) W.s_val[q] = q_ts - (G + aex);  // for later rounds and the window carry\n      const int iu = q > qc ? q_ts + (aex - aex_rs) : q_val + G + aex;  // coordinate at the unit start\n      const int i = iu + adv0;                // ... and at its main token\n      // ---- effects ----\n      uint32_t te = err;\n      if (adv0 > 0 && (iu < 0 || i > n)) te |= DE_INDEX;  // prefix \':\' writes refarr[2 iu + 1 ...] (:75-80)\n      if (kind == 1 && (i < 0 || i + adv > n)) te |= DE_INDEX;\n      if (kind == 2 && (uint32_t)i >= (uint32_t)n) te |= DE_INDEX;\n      if (kind == 3 && (uint32_t)i > (uint32_t)n) te |= DE_INDEX;\n      const int rl = q_read;\n      if (te == 0) {\n        if (kind == 2 && (TM != 3 || a.sub_wins == 0)) odd_sub(i, (int)pay);\n        if (kind == 4 && i >= 0 && i < n) {\n          depth_dec(i);\n          depth_inc(i + olen_e < n ? i + olen_e : n);\n        }\n        if (kind == 3) {\n          atomicOr(hl + (i >> 5), 1u << (i & 31));\n          if (olen_e > kInsInline) push_ovf(a, A + sx + 1, rl, i, olen_e);\n        }\n      }\n      if (TM == 3 && a.sub_wins > 0) {  // substitution events, wave-aggregated per window\n        const bool sev = te == 0 && kind == 2;\n        const int win = i >> kSubWinBits;\n        for (int ww = 0; ww < a.sub_wins; ++ww) {\n          const uint64_t bw = ballot(sev && win == ww);\n          if (!bw) continue;\n          const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)nsub_v, ww);\n          if (sev && win == ww)\n            a.subev[(int64_t)ww * a.subev_cap + sev_base + n0 + lanes_below(bw)] =\n                (uint16_t)(((uint32_t)(i & (kSubWin - 1)) << 2) | pay);\n          if (l == ww) nsub_v += (uint32_t)__popcll(bw);\n        }\n      }\n      const bool ins_inline = kind == 3 && olen_e <= kInsInline && te == 0;\n      const uint64_t bins = ballot(ins_inline);\n      if (ins_inline) {\n        a.ins_raw[ev_base + nev + lanes_below(bins)] = ins_event(i, olen_e, pay, a.read_offset + rl);\n        atomicAdd(bcnt + i / kBW, 1u);\n      }\n      if (last) {  // the read\'s last operation: i_end, downstream check, span\n        const int ia = i + adv;\n        const int ie = ia < 0 ? 0 : (ia > n ? n + 1 : ia);\n        const int dnf = q_iend & (1 << 30);\n        if (dnf && ia > n) te |= DE_INDEX;   // rightIndel(2*i) past the end\n        W.s_iend[q] = ie | dnf;\n        const int ts = q_ts;\n        const int e2 = ie > n ? n : ie;\n        if (ts >= 0 && ts < e2) { depth_inc(ts); depth_dec(e2); }\n      }\n      if (te) flag_read(a, te, rl);\n      G += atot;\n      qc += __popcll(brs);\n      nev += (uint32_t)__popcll(bins);\n    }\n', "    // ---- rounds: two consecutive units per lane (128 per round): the lane's\n    // advances are summed before ONE wave scan, the read-start max-scan keys\n    // on the lane's last start ----\n    int32_t G = 0;  // advances of the window's earlier rounds\n    int qc = 0;     // read starts of the window's earlier rounds\n    struct UnitD { int s0, sx, pl, adv0, adv, kind, olen_e; uint32_t pay, err; bool is_rs, last; };\n    const uint32_t* b32 = reinterpret_cast<const uint32_t*>(W.stage);\n    auto decode = [&](uint32_t e0, uint32_t e1, bool v) {\n      UnitD u;\n      const int s0 = (int)(e0 & 0xfffu);         // unit start\n      const int pl = (int)((e0 >> 12) & 7u);     // ':' operand length of a unit's prefix (0: none)\n      const int sx = pl ? s0 + pl + 1 : s0;      // the unit's main token\n      const bool lfar = v && ((e1 & 0x7fffu) == kFar);\n      const int64_t ex64 = lfar ? C - A : (int64_t)(e1 & 0xfffu);  // far: the token ends at C (beyond the window)\n      const int ex = (int)(ex64 - sx - 1 < kAdvCap ? ex64 : sx + 1 + kAdvCap);\n      const bool last = v && (e1 >> 15);\n      // fast decode from the staged bytes: op, then 4 operand bytes\n      const int a4 = sx >> 2;\n      const uint32_t sh = (uint32_t)(sx & 3);\n      const uint32_t d0 = b32[a4], d1 = b32[a4 + 1], d2 = b32[a4 + 2];\n      const uint32_t x0 = __builtin_amdgcn_alignbyte(d1, d0, sh);\n      const uint32_t x1 = __builtin_amdgcn_alignbyte(d2, d1, sh);\n      const uint32_t op = x0 & 0xffu;\n      const uint32_t w0 = __builtin_amdgcn_alignbyte(x1, x0, 1u);\n      const int olen = ex - sx - 1;\n      const bool colon = op == ':', star = op == '*', plus = op == '+', minus = op == '-';\n      const bool spec = colon | star | plus | minus | (op == 'Z');\n      const bool act = v & spec & ((olen > 0) | last);  // empty operand: skipped unless last (:309, :320)\n      const int ol4 = olen < 0 ? 0 : (olen > 4 ? 4 : olen);\n      const uint32_t vm = ol4 == 4 ? 0xffffffffu : ((1u << (8 * ol4)) - 1u);  // operand bytes in w0\n      const bool pre = pl != 0;\n      const int pa = (s0 + 1) >> 2;\n      const uint32_t pw = __builtin_amdgcn_alignbyte(b32[pa + 1], b32[pa], (uint32_t)((s0 + 1) & 3));\n      const int cl = pre ? pl : (colon ? ol4 : 0);\n      const uint32_t cw = pre ? pw : w0;\n      const uint32_t cvm = cl == 4 ? 0xffffffffu : ((1u << (8 * cl)) - 1u);\n      const uint32_t Tx = cw ^ 0x30303030u;\n      const bool cdig = ((((Tx & 0x7F7F7F7Fu) + 0x76767676u) | Tx) & 0x80808080u & cvm) == 0;\n      uint32_t X = cl == 0 ? 0u : (Tx & cvm & 0x0F0F0F0Fu) << (8 * (4 - cl));\n      X = mul2561(X) >> 8;\n      X = ((X & 0x00FF00FFu) * 6553601u) >> 16;\n      const int adv_c = (int)(X & 0xffffu);\n      int adv0 = pre ? adv_c : 0;\n      const bool dig_ok = (olen >= 1) & (olen <= 4) & cdig;  // main ':' token\n      const uint32_t lc = w0 | 0x20202020u;\n      const uint32_t hh = (lc >> 1) & 0x03030303u;\n      const uint32_t bad = lc ^ __builtin_amdgcn_perm(0u, 0x67746361u, hh);\n      const uint32_t codes = ((hh & 0x01010101u) << 1) | ((hh >> 1) & 0x01010101u);  // dict order A0 T1 C2 G3\n      const int shl = 8 * ((olen - 1) & 3);\n      const bool last_ok = ((bad >> shl) & 0xffu) == 0;  // '*': written base = operand[-1] (:96)\n      uint32_t pk = codes;\n      pk = (pk | (pk >> 6)) & 0x000f000fu;\n      pk = (pk | (pk >> 12)) & 0xffu;\n      const uint32_t mstar = 0u - (uint32_t)star;\n      uint32_t pay = (mstar & ((codes >> shl) & 3u)) | (~mstar & (pk & ((1u << (2 * ol4)) - 1u)));\n      const bool slow = lfar | (pre & !cdig) | (act & ((colon & !dig_ok) | ((star | plus) & (olen > 4))));\n      const int kop = ((int)star << 1) | ((int)plus * 3) | ((int)minus << 2);  // exclusive classes\n      const int mcol = -(int)colon;\n      int kind = (-(int)act) & ((mcol & (int)(adv_c > 0)) | (~mcol & (-(int)(olen > 0) & kop)));\n      int adv = (-(int)(kind == 1) & adv_c) | (int)(kind == 2) | (-(int)(kind == 4) & (olen < kAdvCap ? olen : kAdvCap));\n      uint32_t err = (v & !spec) ? DE_OP : 0u;  // cs does not start with an operator (:100-102)\n      if (act & star & (olen == 0)) err |= DE_INDEX;  // operand[-1] of '' (:96)\n      if ((kind == 2) & !last_ok) err |= DE_KEY;\n      if ((kind == 3) & ((bad & vm) != 0)) err |= DE_KEY;\n      int olen_e = olen;\n      if (slow) {  // rare: decode from HBM\n        const int64_t s = A + sx, e = A + ex64;\n        const TokInfo ti = analyze_long(a.cs, s, e, last);\n        adv = ti.adv; kind = ti.kind; pay = ti.pay; err = ti.err;\n        olen_e = (int)(e - s - 1 < kAdvCap ? e - s - 1 : kAdvCap);\n        if (pl) {\n          const TokInfo tp = analyze_long(a.cs, A + s0, s, false);\n          adv0 = tp.adv;\n          err |= tp.err;\n        }\n      }\n      u.s0 = s0; u.sx = sx; u.pl = pl; u.adv0 = adv0; u.adv = adv; u.kind = kind; u.olen_e = olen_e;\n      u.pay = pay; u.err = err; u.is_rs = v && (e0 >> 15); u.last = last;\n      return u;\n    };\n    // effects of one unit at coordinate iu (unit start); wave-uniform call\n    auto effects = [&](const UnitD& u, int iu, int q, int32_t q_ts, int32_t q_read, int32_t q_iend) {\n      const int adv0 = u.adv0, adv = u.adv, kind = u.kind, olen_e = u.olen_e;\n      const uint32_t pay = u.pay;\n      const int i = iu + adv0;                // coordinate at the main token\n      uint32_t te = u.err;\n      if (adv0 > 0 && (iu < 0 || i > n)) te |= DE_INDEX;  // prefix ':' writes refarr[2 iu + 1 ...] (:75-80)\n      if (kind == 1 && (i < 0 || i + adv > n)) te |= DE_INDEX;\n      if (kind == 2 && (uint32_t)i >= (uint32_t)n) te |= DE_INDEX;\n      if (kind == 3 && (uint32_t)i > (uint32_t)n) te |= DE_INDEX;\n      const int rl = q_read;\n      if (te == 0) {\n        if (kind == 2 && (TM != 3 || a.sub_wins == 0)) odd_sub(i, (int)pay);\n        if (kind == 4 && i >= 0 && i < n) {\n          depth_dec(i);\n          depth_inc(i + olen_e < n ? i + olen_e : n);\n        }\n        if (kind == 3) {\n          atomicOr(hl + (i >> 5), 1u << (i & 31));\n          if (olen_e > kInsInline) push_ovf(a, A + u.sx + 1, rl, i, olen_e);\n        }\n      }\n      if (TM == 3 && a.sub_wins > 0) {  // substitution events, wave-aggregated per window\n        const bool sev = te == 0 && kind == 2;\n        const int win = i >> kSubWinBits;\n        for (int ww = 0; ww < a.sub_wins; ++ww) {\n          const uint64_t bw = ballot(sev && win == ww);\n          if (!bw) continue;\n          const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)nsub_v, ww);\n          if (sev && win == ww)\n            a.subev[(int64_t)ww * a.subev_cap + sev_base + n0 + lanes_below(bw)] =\n                (uint16_t)(((uint32_t)(i & (kSubWin - 1)) << 2) | pay);\n          if (l == ww) nsub_v += (uint32_t)__popcll(bw);\n        }\n      }\n      const bool ins_inline = kind == 3 && olen_e <= kInsInline && te == 0;\n      const uint64_t bins = ballot(ins_inline);\n      if (ins_inline) {\n        a.ins_raw[ev_base + nev + lanes_below(bins)] = ins_event(i, olen_e, pay, a.read_offset + rl);\n        atomicAdd(bcnt + i / kBW, 1u);\n      }\n      if (u.last) {  // the read's last operation: i_end, downstream check, span\n        const int ia = i + adv;\n        const int ie = ia < 0 ? 0 : (ia > n ? n + 1 : ia);\n        const int dnf = q_iend & (1 << 30);\n        if (dnf && ia > n) te |= DE_INDEX;   // rightIndel(2*i) past the end\n        W.s_iend[q] = ie | dnf;\n        const int ts = q_ts;\n        const int e2 = ie > n ? n : ie;\n        if (ts >= 0 && ts < e2) { depth_inc(ts); depth_dec(e2); }\n      }\n      if (te) flag_read(a, te, rl);\n      nev += (uint32_t)__popcll(bins);\n    };\n    constexpr int kTokEnd = tok_cap<WIN>() + 2 + 64 - 1;  // last readable entry\n    for (int t0 = 0; t0 < T; t0 += 128) {\n      const int tA = t0 + 2 * l;\n      const bool vA = tA < T, vB = tA + 1 < T;\n      const uint32_t r0 = W.tok[min(tA, kTokEnd)], r1 = W.tok[min(tA + 1, kTokEnd)], r2 = W.tok[min(tA + 2, kTokEnd)];\n      const uint32_t eA0 = vA ? r0 : 0u, eA1 = vA ? r1 : 0u, eB0 = vB ? r1 : 0u, eB1 = vB ? r2 : 0u;\n      const bool rsA = vA && (eA0 >> 15), rsB = vB && (eB0 >> 15);\n      const uint64_t bA = ballot(rsA), bB = ballot(rsB);\n      const int qA = qc + lanes_below(bA) + lanes_below(bB) + (rsA ? 1 : 0);\n      const int qB = qA + (rsB ? 1 : 0);\n      // the reads' slots, loaded before the decode\n      const int32_t vA_val = W.s_val[qA], vA_ts = W.s_ts[qA], vA_read = W.s_read[qA], vA_iend = W.s_iend[qA];\n      const int32_t vB_val = W.s_val[qB], vB_ts = W.s_ts[qB], vB_read = W.s_read[qB], vB_iend = W.s_iend[qB];\n      const UnitD uA = decode(eA0, eA1, vA);\n      const UnitD uB = decode(eB0, eB1, vB);\n      // ---- coordinates ----\n      const int advA = uA.adv0 + uA.adv, advB = uB.adv0 + uB.adv;  // each <= 2^21: 128 units stay < 2^31\n      const int sum2 = advA + advB;\n      const int ainc = wave_scan_i32(sum2);\n      const int aexA = ainc - sum2, aexB = aexA + advA;  // advances of the round before each unit\n      const int atot = wave_last_i32(ainc);\n      // the latest read start at or before each unit: aex never decreases, so\n      // it is a max-scan of the lanes' last starts (DPP), shifted for unit A\n      const int key = rsB ? aexB : (rsA ? aexA : 0);\n      const int kinc = wave_scan_max_i32(key);\n      const int kprev = (int)from_lane_below((uint32_t)kinc);  // lanes below this one\n      const int krsA = rsA ? aexA : kprev;\n      const int krsB = rsB ? aexB : krsA;\n      if (rsA) W.s_val[qA] = vA_ts - (G + aexA);  // for later rounds and the window carry\n      if (rsB) W.s_val[qB] = vB_ts - (G + aexB);\n      const int iuA = qA > qc ? vA_ts + (aexA - krsA) : vA_val + G + aexA;  // coordinates at the unit starts\n      const int iuB = qB > qc ? vB_ts + (aexB - krsB) : vB_val + G + aexB;\n      effects(uA, iuA, qA, vA_ts, vA_read, vA_iend);\n      effects(uB, iuB, qB, vB_ts, vB_read, vB_iend);\n      G += atot;\n      qc += __popcll(bA) + __popcll(bB);\n    }\n")]
PATCHES["fl_store"] = [("""        if (wr >= 0 && wr < kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
        else atomicAdd(a.rows + row * 4 + code, 1u);
      }""", """        if (wr >= 0 && wr < kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
        else a.rows[row * 4 + code] = 1u;
      }""")]
PATCHES["fl_lds2"] = [("""        if (wr >= 0 && wr < kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
        else atomicAdd(a.rows + row * 4 + code, 1u);
      }""", """        if (wr >= 0 && wr < kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
        else atomicAdd(wn + ((uint32_t)row & 255u) * 5 + code, 1u);
      }""")]
PATCHES["l_nounits"] = [("""  for (int64_t u = blockIdx.x; u < nunits; u += gridDim.x) {
    for (int k = threadIdx.x; k < kBW * kMs; k += blockDim.x) Ml[k] = 0;""", """  for (int64_t u = blockIdx.x; u < nunits && a.N < 0; u += gridDim.x) {
    for (int k = threadIdx.x; k < kBW * kMs; k += blockDim.x) Ml[k] = 0;""")]
PATCHES["l_noflank"] = [("""  for (int64_t r0 = fb * blockDim.x; r0 < a.N; r0 += nthreads) {
    const int64_t r = r0 + threadIdx.x;""", """  for (int64_t r0 = fb * blockDim.x; r0 < a.N && a.N < 0; r0 += nthreads) {
    const int64_t r = r0 + threadIdx.x;""")]
PATCHES["l_noevt"] = [("""#pragma unroll
    for (int q = 0; q < kEPT; ++q) {
      const uint32_t ev = evs[q];
      if (ev == ~0u) continue;""", """#pragma unroll
    for (int q = 0; q < kEPT; ++q) {
      const uint32_t ev = evs[q];
      if (ev == ~0u || a.N > 0) continue;""")]
PATCHES["ept8"] = [("constexpr int kEPT = 16;", "constexpr int kEPT = 8;")]
PATCHES["ept12"] = [("constexpr int kEPT = 16;", "constexpr int kEPT = 12;")]
PATCHES["ept10"] = [("constexpr int kEPT = 16;", "constexpr int kEPT = 10;")]
PATCHES["ept14"] = [("constexpr int kEPT = 16;", "constexpr int kEPT = 14;")]
FLAGS = {
  "s_ilp": ["-mllvm", "-amdgpu-sched-strategy=max-ilp"],
  "s_iilp": ["-mllvm", "-amdgpu-sched-strategy=iterative-ilp"],
  "s_mmc": ["-mllvm", "-amdgpu-sched-strategy=max-memory-clause"],
  "s_minreg": ["-mllvm", "-amdgpu-sched-strategy=iterative-minreg"],
}
for _k in FLAGS: PATCHES[_k] = []
PATCHES["w5"] = [("__global__ __launch_bounds__(kMaxPW * 64) void K_parse(ParseArgs a) {",
                  "__global__ __launch_bounds__(kMaxPW * 64) __attribute__((amdgpu_waves_per_eu(5))) void K_parse(ParseArgs a) {"),
                 ("    const int max_waves_cu = 16;  // VGPR budget of K_parse (<= 128 VGPRs -> 4 waves per SIMD)",
                  "    const int max_waves_cu = 20;  // VGPR budget of K_parse (<= 96 VGPRs -> 5 waves per SIMD)"),
                 ("      for (int nw : {16, 12, 8}) {", "      for (int nw : {16, 12, 10, 8}) {")]
PATCHES["w5only"] = [PATCHES["w5"][0]]
PATCHES["flat"] = [("""      uint32_t te = err;
      if (adv0 > 0 && (iu < 0 || i > n)) te |= DE_INDEX;  // prefix ':' writes refarr[2 iu + 1 ...] (:75-80)
      if (kind == 1 && (i < 0 || i + adv > n)) te |= DE_INDEX;
      if (kind == 2 && (uint32_t)i >= (uint32_t)n) te |= DE_INDEX;
      if (kind == 3 && (uint32_t)i > (uint32_t)n) te |= DE_INDEX;
      const int rl = q_read;
      if (te == 0) {
        if (kind == 2 && (TM != 3 || a.sub_wins == 0)) odd_sub(i, (int)pay);
        if (kind == 4 && i >= 0 && i < n) {
          depth_dec(i);
          depth_inc(i + olen_e < n ? i + olen_e : n);
        }
        if (kind == 3) {
          atomicOr(hl + (i >> 5), 1u << (i & 31));
          if (olen_e > kInsInline) push_ovf(a, A + sx + 1, rl, i, olen_e);
        }
      }""", """      // data errors and effects as flat predicates (no nested exec-mask regions)
      const bool bad_i = ((adv0 > 0) & ((iu < 0) | (i > n))) | ((kind == 1) & ((i < 0) | (i + adv > n))) |
                         ((kind == 2) & ((uint32_t)i >= (uint32_t)n)) | ((kind == 3) & ((uint32_t)i > (uint32_t)n));
      uint32_t te = err | (bad_i ? DE_INDEX : 0u);
      const int rl = q_read;
      const bool ok = te == 0;
      if (ok & (kind == 2) & (TM != 3 || a.sub_wins == 0)) odd_sub(i, (int)pay);
      const bool del = ok & (kind == 4) & (i >= 0) & (i < n);
      if (del) {
        depth_dec(i);
        depth_inc(i + olen_e < n ? i + olen_e : n);
      }
      if (ok & (kind == 3)) atomicOr(hl + (i >> 5), 1u << (i & 31));
      if (ok & (kind == 3) & (olen_e > kInsInline)) push_ovf(a, A + sx + 1, rl, i, olen_e);""")]
PATCHES["flat2"] = PATCHES["flat"] + [("""      uint32_t err = (v & !spec) ? DE_OP : 0u;  // cs does not start with an operator (:100-102)
      if (act & star & (olen == 0)) err |= DE_INDEX;  // operand[-1] of '' (:96)
      if ((kind == 2) & !last_ok) err |= DE_KEY;
      if ((kind == 3) & ((bad & vm) != 0)) err |= DE_KEY;""",
"""      uint32_t err = ((v & !spec) ? DE_OP : 0u) |                        // cs does not start with an operator (:100-102)
                     ((act & star & (olen == 0)) ? DE_INDEX : 0u) |      // operand[-1] of '' (:96)
                     ((((kind == 2) & !last_ok) | ((kind == 3) & ((bad & vm) != 0))) ? DE_KEY : 0u);"""),
("""      if (last) {  // the read's last operation: i_end, downstream check, span
        const int ia = i + adv;
        const int ie = ia < 0 ? 0 : (ia > n ? n + 1 : ia);
        const int dnf = q_iend & (1 << 30);
        if (dnf && ia > n) te |= DE_INDEX;   // rightIndel(2*i) past the end
        W.s_iend[q] = ie | dnf;
        const int ts = q_ts;
        const int e2 = ie > n ? n : ie;
        if (ts >= 0 && ts < e2) { depth_inc(ts); depth_dec(e2); }
      }""", """      {  // the read's last operation: i_end, downstream check, span
        const int ia = i + adv;
        const int ie = ia < 0 ? 0 : (ia > n ? n + 1 : ia);
        const int dnf = q_iend & (1 << 30);
        te |= (last & (dnf != 0) & (ia > n)) ? DE_INDEX : 0u;   // rightIndel(2*i) past the end
        if (last) W.s_iend[q] = ie | dnf;
        const int ts = q_ts;
        const int e2 = ie > n ? n : ie;
        if (last & (ts >= 0) & (ts < e2)) { depth_inc(ts); depth_dec(e2); }
      }""")]
PATCHES["sval"] = [
("      const int32_t q_val = W.s_val[q], q_ts = W.s_ts[q], q_read = W.s_read[q], q_iend = W.s_iend[q];",
 "      const int32_t q_ts = W.s_ts[q], q_read = W.s_read[q], q_iend = W.s_iend[q];"),
("""      const int aex_rs = wave_scan_max_i32(is_rs ? aex : 0);
      if (is_rs) W.s_val[q] = q_ts - (G + aex);  // for later rounds and the window carry
      const int iu = q > qc ? q_ts + (aex - aex_rs) : q_val + G + aex;  // coordinate at the unit start""",
"""      // a read starting in this round writes its base into the slot first;
      // every lane then reads its read's base back (one LDS round trip instead
      // of a max-scan): i = base + advances before the unit
      if (is_rs) W.s_val[q] = q_ts - (G + aex);  // for later rounds and the window carry
      wave_sync_lds();
      const int iu = W.s_val[q] + G + aex;  // coordinate at the unit start""")]
PATCHES["bperm"] = [("""      const int aex_rs = wave_scan_max_i32(is_rs ? aex : 0);""",
"""      // the latest read-start lane <= this one (ballot bits), its aex by one permute
      const uint64_t m_rs = brs & (l == 63 ? ~0ull : ((2ull << l) - 1ull));
      const int j_rs = m_rs ? 63 - __clzll((long long)m_rs) : 0;
      const int aex_j = __shfl(aex, j_rs, 64);
      const int aex_rs = m_rs ? aex_j : 0;""")]
PATCHES["ex32"] = [("""      const int64_t ex64 = lfar ? C - A : (int64_t)(e1 & 0xfffu);  // far: the token ends at C (beyond the window)
      const int ex = (int)(ex64 - sx - 1 < kAdvCap ? ex64 : sx + 1 + kAdvCap);""",
"""      // far: the token ends at C (beyond the window); 32-bit here (far_c saturates
      // at 2^30 > kAdvCap + the window), 64-bit only on the slow path
      const int ex32 = lfar ? far_c : (int)(e1 & 0xfffu);
      const int ex = ex32 - sx - 1 < kAdvCap ? ex32 : sx + 1 + kAdvCap;"""),
("""        const int64_t s = A + sx, e = A + ex64;""", """        const int64_t s = A + sx, e = A + (lfar ? C - A : (int64_t)(e1 & 0xfffu));"""),
("""    int32_t G = 0;  // advances of the window's earlier rounds""", """    const int far_c = (int)(C - A < (1 << 30) ? C - A : (1 << 30));  // wave-uniform
    int32_t G = 0;  // advances of the window's earlier rounds""")]
PATCHES["capskip"] = [("""      const int cb = __popc(m);
      const int inc = wave_scan_i32(cb);
      if (wave_last_i32(inc) > tok_cap<WIN>()) {""", """      const int cb = __popc(m);
      // at most tok_cap / 64 boundaries in every lane: no cut (the usual case, no scan)
      const bool may = ballot(cb > tok_cap<WIN>() / 64) != 0;
      const int inc = may ? wave_scan_i32(cb) : 0;
      if (may && wave_last_i32(inc) > tok_cap<WIN>()) {""")]
PATCHES["subptr"] = [("""        const int win = i >> kSubWinBits;
        for (int ww = 0; ww < a.sub_wins; ++ww) {
          const uint64_t bw = ballot(sev && win == ww);
          if (!bw) continue;
          const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)nsub_v, ww);
          if (sev && win == ww)
            a.subev[(int64_t)ww * a.subev_cap + sev_base + n0 + lanes_below(bw)] =
                (uint16_t)(((uint32_t)(i & (kSubWin - 1)) << 2) | pay);
          if (l == ww) nsub_v += (uint32_t)__popcll(bw);
        }""", """        const int win = i >> kSubWinBits;
        uint16_t* wp = a.subev + sev_base;  // window ww's region of this wave
        for (int ww = 0; ww < a.sub_wins; ++ww, wp += a.subev_cap) {
          const bool mine = sev && win == ww;
          const uint64_t bw = ballot(mine);
          if (!bw) continue;
          const uint32_t n0 = (uint32_t)__builtin_amdgcn_readlane((int)nsub_v, ww);
          if (mine) wp[n0 + lanes_below(bw)] = (uint16_t)(((uint32_t)(i & (kSubWin - 1)) << 2) | pay);
          if (l == ww) nsub_v += (uint32_t)__popcll(bw);
        }""")]
PATCHES["micro1"] = [("""      const int ex32 = lfar ? far_c : (int)(e1 & 0xfffu);
      const int ex = ex32 - sx - 1 < kAdvCap ? ex32 : sx + 1 + kAdvCap;""",
"""      const int ex = lfar ? (far_c - sx - 1 < kAdvCap ? far_c : sx + 1 + kAdvCap) : (int)(e1 & 0xfffu);"""),
("""        a.ins_raw[ev_base + nev + lanes_below(bins)] = ins_event(i, olen_e, pay, a.read_offset + rl);""",
 """        evp[nev + lanes_below(bins)] = ins_event(i, olen_e, pay, a.read_offset + rl);"""),
("""  uint32_t nev = 0;                                       // events written (wave-uniform)""",
 """  uint32_t nev = 0;                                       // events written (wave-uniform)
  uint64_t* const evp = a.ins_raw + ev_base;""")]
PATCHES["l32"] = [("""      const int64_t rg = a.read_offset + s_r0[jsq[q]] + (ev >> 16);""",
"""      const int32_t rg = (int32_t)a.read_offset + s_r0[jsq[q]] + (int32_t)(ev >> 16);  // global reads < 2^30"""),
("""      if (lb > la) k += vl ? lower_bound_i32(s_vals, la - v0, lb - v0, (int32_t)rg) - (la - v0)
                           : lower_bound_i32(a.vals_out, la, lb, (int32_t)rg) - la;""",
"""      if (lb > la) {
        if (vl) {  // 32-bit search of the staged RIGHT reads
          int lo = la - v0, hi = lb - v0;
          const int l0 = lo;
          while (lo < hi) {
            const int mid = (lo + hi) >> 1;
            if (s_vals[mid] < rg) lo = mid + 1; else hi = mid;
          }
          k += lo - l0;
        } else {
          k += lower_bound_i32(a.vals_out, la, lb, rg) - la;
        }
      }""")]
PATCHES["l32b"] = PATCHES["l32"] + [("""      int64_t k = s_roff[p];
      if (lb > la) {""", """      int32_t k = s_roff[p];  // run of the event within its gap
      if (lb > la) {"""),
("""        atomicMax(a.M + s_rs[p] + g + k, L);
        uint32_t* rt = a.runt + (s_rs[p] + g + k) * 16;""", """        atomicMax(a.M + s_rs[p] + g + (int64_t)k, L);
        uint32_t* rt = a.runt + (s_rs[p] + g + (int64_t)k) * 16;""")]
PATCHES["l4"] = PATCHES["l32b"] + [("""        for (int j = 0; j < L; ++j) atomicAdd(tp + 4 * (L - 1 - j) + (int)((ev >> (2 * j)) & 3u), 1u);
      } else {""", """#pragma unroll
        for (int j = 0; j < kInsInline; ++j)  // straight-line: bases j < L
          if (j < L) atomicAdd(tp + 4 * (L - 1 - j) + (int)((ev >> (2 * j)) & 3u), 1u);
      } else {""")]
PATCHES["f32"] = [("""      for (int x = tid; x < cn; x += blockDim.x) {
        const uint32_t word = bm[x >> 5];
        const int o = wpre[x >> 5] + __popc(word & (0xffffffffu >> (31 - (x & 31))));  // owner: starts <= x
        const int32_t rw = t_row[o];
        if (rw < 0) continue;
        const int64_t row = (int64_t)rw + (c0 + x - t_start[o]);
        const int code = code_exact(stage[x + sh0]);
        if (code < 0) { lerr |= DE_KEY; const int64_t rr = r0 + t_read[o]; lread = rr < lread ? rr : lread; continue; }
        const int64_t wr = row - w0;
        if (wr >= 0 && wr < kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
        else atomicAdd(a.rows + row * 4 + code, 1u);
      }""", """      // 32-bit: rows < row_cap < 2^31, a block's flank bytes < 2^31
      const int cn32 = (int)cn, c032 = (int)c0;
      const int32_t w032 = w0 >= 0 ? (int32_t)w0 : -(1 << 30);  // no window: never a hit
      for (int x = tid; x < cn32; x += blockDim.x) {
        const uint32_t word = bm[x >> 5];
        const int o = wpre[x >> 5] + __popc(word & (0xffffffffu >> (31 - (x & 31))));  // owner: starts <= x
        const int32_t rw = t_row[o];
        if (rw < 0) continue;
        const int32_t row = rw + (c032 + x - t_start[o]);
        const int code = code_exact(stage[x + sh0]);
        if (code < 0) { lerr |= DE_KEY; const int64_t rr = r0 + t_read[o]; lread = rr < lread ? rr : lread; continue; }
        const uint32_t wr = (uint32_t)(row - w032);
        if (wr < (uint32_t)kWinRows) atomicAdd(wn + wr * 5 + code, 1u);
        else atomicAdd(a.rows + (int64_t)row * 4 + code, 1u);
      }""")]
PATCHES["epi32"] = [("""  return ((uint32_t)raw & 0x3ffu) | ((gap % (uint32_t)kBW) << 10) | ((uint32_t)((int64_t)(raw >> 32) - rg0) << 16);""",
"""  return ((uint32_t)raw & 0x3ffu) | ((gap % (uint32_t)kBW) << 10) | (((uint32_t)(raw >> 32) - (uint32_t)rg0) << 16);""")]
PATCHES["i32"] = [("""    const int64_t t0 = (int64_t)a.right_start[g] + g, t1 = (int64_t)a.right_start[g + 1] + g + 1;
    const int64_t top = (int64_t)a.row_base[g] + a.lo_f[g] - 1;
    const bool excl = no_ovf && t1 - t0 == 1;
    for (int64_t t = t0; t < t1; ++t) {
      uint4* rt = reinterpret_cast<uint4*>(a.runt + t * 16);""", """    // 32-bit: runs < n_reads_global + gaps < 2^31, rows < 2^31
    const int32_t gi = (int32_t)g;
    const int32_t t0 = a.right_start[g] + gi, t1 = a.right_start[g + 1] + gi + 1;
    const int32_t top = a.row_base[g] + a.lo_f[g] - 1;
    const bool excl = no_ovf && t1 - t0 == 1;
    for (int32_t t = t0; t < t1; ++t) {
      uint4* rt = reinterpret_cast<uint4*>(a.runt) + 4 * (int64_t)t;"""),
("""      const int64_t rtop = top + a.hiR[t];
#pragma unroll
      for (int bi = 0; bi < 4; ++bi) {
        uint32_t* row = a.rows + (rtop - bi) * 4;""", """      const int32_t rtop = top + a.hiR[t];
#pragma unroll
      for (int bi = 0; bi < 4; ++bi) {
        uint32_t* row = a.rows + (int64_t)(rtop - bi) * 4;""")]
PATCHES["evlocal"] = [
("""        a.ins_raw[ev_base + nev + lanes_below(bins)] = ins_event(i, olen_e, pay, a.read_offset + rl);""",
 """        a.ins_raw[ev_base + nev + lanes_below(bins)] = ins_event(i, olen_e, pay, rl);"""),
("""  const int64_t rg0 = a.read_offset + r0;  // the workgroup's first (global) read""",
 """  const int64_t rg0 = r0;  // the workgroup's first read (raw events hold launch-local reads)""")]
PATCHES["tok2"] = [("""      const uint32_t t0r = W.tok[t], t1r = W.tok[t + 1];  // in bounds for every lane (+64 padding)""",
"""      // entries t, t + 1 from one ds_read2 of the dwords holding them (in bounds: +64 padding)
      const uint32_t* tk32 = reinterpret_cast<const uint32_t*>(W.tok);
      const uint32_t da = tk32[t >> 1], db = tk32[(t >> 1) + 1];
      const bool odd = (t & 1) != 0;
      const uint32_t t0r = odd ? (da >> 16) : (da & 0xffffu);
      const uint32_t t1r = odd ? (db & 0xffffu) : (da >> 16);""")]
PATCHES["cmp2"] = [("""      uint32_t m = tu;
      while (m) {
        const int k = __ffs(m) - 1;
        m &= m - 1;
        W.tok[idx++] = (uint16_t)((uint32_t)(base + k) | (((pl0 >> k) & 1u) << 12) | (((pl1 >> k) & 1u) << 13) |
                                  (((p5 >> k) & 1u) << 14) | (((ra_own >> k) & 1u) << 15));
      }""", """      uint32_t m = tu;
      auto entry = [&](int k) {
        return (uint16_t)((uint32_t)(base + k) | (((pl0 >> k) & 1u) << 12) | (((pl1 >> k) & 1u) << 13) |
                          (((p5 >> k) & 1u) << 14) | (((ra_own >> k) & 1u) << 15));
      };
      while (m) {  // two entries per trip (half the loop control)
        const int k1 = __ffs(m) - 1;
        m &= m - 1;
        W.tok[idx] = entry(k1);
        if (m) {
          const int k2 = __ffs(m) - 1;
          m &= m - 1;
          W.tok[idx + 1] = entry(k2);
        }
        idx += 2;
      }""")]
PATCHES["mdepth"] = [("""      const bool del = ok & (kind == 4) & (i >= 0) & (i < n);
      if (del) {
        depth_dec(i);
        depth_inc(i + olen_e < n ? i + olen_e : n);
      }
""", ""),
("""      if (last) {  // the read's last operation: i_end, downstream check, span
        const int ia = i + adv;
        const int ie = ia < 0 ? 0 : (ia > n ? n + 1 : ia);
        const int dnf = q_iend & (1 << 30);
        if (dnf && ia > n) te |= DE_INDEX;   // rightIndel(2*i) past the end
        W.s_iend[q] = ie | dnf;
        const int ts = q_ts;
        const int e2 = ie > n ? n : ie;
        if (ts >= 0 && ts < e2) { depth_inc(ts); depth_dec(e2); }
      }""", """      {  // depth differences: a deletion (-1 at i, +1 at its end) and / or, at the
         // read's last operation, its span (+1 at tstart, -1 at its end): one
         // exec region for the usual single update, a second for both
        const int ia = i + adv;
        const int ie = ia < 0 ? 0 : (ia > n ? n + 1 : ia);
        const int dnf = q_iend & (1 << 30);
        const int ts = q_ts;
        const int e2 = ie > n ? n : ie;
        const bool del = ok & (kind == 4) & (i >= 0) & (i < n);
        const bool span = last & (ts >= 0) & (ts < e2);
        if (del | span) {
          depth_dec(del ? i : e2);
          depth_inc(del ? (i + olen_e < n ? i + olen_e : n) : ts);
        }
        if (del & span) { depth_inc(ts); depth_dec(e2); }
        if (last) {  // the read's last operation: i_end, downstream check
          if (dnf && ia > n) te |= DE_INDEX;   // rightIndel(2*i) past the end
          W.s_iend[q] = ie | dnf;
        }
      }""")]
