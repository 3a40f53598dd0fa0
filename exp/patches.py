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
