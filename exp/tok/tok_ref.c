// CPU statement of the prototype tokenizer's unit stream (exp/tok/k_tok.hip),
// the checker of that experiment only.  Tokens follow the reference's cs loop
// (src/mapped_paf_read_parser.py:307-318): a token starts at every special
// character (':', 'Z', '+', '-', '*') and at every read start; it runs to the
// next token start.  A ':' token directly followed (same read) by a non-':'
// special token is absorbed into that token's unit, so a unit is
// "match run, then one operation" -- the unit K_parse already decodes.
//
// unit word: op(3) | rs(1) << 3 | oplen(6) << 4 | payload(8) << 10 | match(14) << 18
//   op: 0 ':' alone, 1 '*', 2 '+', 3 '-', 4 'Z', 5 read start on a non-special byte
//   rs: the unit's first token starts a read
//   oplen: operand bytes of the operation token (capped at 63)
//   payload: 2-bit codes ((b >> 1) & 3) of its first 4 operand bytes
//   match: the absorbed (or lone) ':' operand as a number; 16383 = escape
//          (not 1-8 digits, or >= 16383): a consumer re-reads those bytes
// Units are emitted in byte order (out[], compact); wcount[w] counts those
// emitted at bytes [w S, (w + 1) S) -- the kernel's per-wave regions.
#include <stdint.h>
#include <string.h>

static int special(uint8_t c) { return c == ':' || c == 'Z' || c == '+' || c == '-' || c == '*'; }
static uint32_t opcode(uint8_t c) {
  switch (c) {
    case ':': return 0;
    case '*': return 1;
    case '+': return 2;
    case '-': return 3;
    case 'Z': return 4;
    default: return 5;
  }
}
static uint32_t colon_value(const uint8_t* cs, int64_t s, int64_t e) {
  const int64_t nd = e - s - 1;
  if (nd < 1 || nd > 8) return 16383;
  uint32_t v = 0;
  for (int64_t k = s + 1; k < e; ++k) {
    if (cs[k] < '0' || cs[k] > '9') return 16383;
    v = v * 10 + (cs[k] - '0');
  }
  return v >= 16383 ? 16383 : v;
}
static uint32_t op_fields(const uint8_t* cs, int64_t s, int64_t e) {
  const int64_t ol = e - s - 1;
  uint32_t pay = 0;
  for (int k = 0; k < 4 && k < ol; ++k) pay |= (uint32_t)((cs[s + 1 + k] >> 1) & 3) << (2 * k);
  return (uint32_t)(ol > 63 ? 63 : ol) << 4 | pay << 10;
}

// returns the number of units (out: compact, in byte order)
int64_t tok_ref(const uint8_t* cs, int64_t B, const int64_t* cs_off, int64_t N, int64_t S, uint32_t* out,
                uint32_t* wcount, int64_t nwaves) {
  memset(wcount, 0, sizeof(uint32_t) * (size_t)nwaves);
  int64_t total = 0, r = 0;
  // token list on the fly: s = current token, its successor found by scanning
  int64_t s = -1;
  for (int64_t p = 0; p < B; ++p) {
    while (r < N && cs_off[r] < p) ++r;
    const int rs = r < N && cs_off[r] == p;
    if (special(cs[p]) || rs) { s = p; break; }
  }
  int64_t prev = -1;
  int prev_rs = 0;
  while (s >= 0 && s < B) {
    while (r < N && cs_off[r] < s) ++r;
    const int rs = r < N && cs_off[r] == s;
    int64_t e = s + 1, r2 = r;
    for (; e < B; ++e) {
      while (r2 < N && cs_off[r2] < e) ++r2;
      if (special(cs[e]) || (r2 < N && cs_off[r2] == e)) break;
    }
    const int nrs = e < B && r2 < N && cs_off[r2] == e;
    const uint8_t op = cs[s];
    int emit = 0;
    uint32_t word = 0;
    if (op == ':') {
      const int absorbed = e < B && special(cs[e]) && cs[e] != ':' && !nrs;
      if (!absorbed) { emit = 1; word = (uint32_t)rs << 3 | colon_value(cs, s, e) << 18; }
    } else if (special(op)) {
      const int merged = prev >= 0 && cs[prev] == ':' && !rs;
      const uint32_t m = merged ? colon_value(cs, prev, s) : 0;
      const int urs = merged ? prev_rs : rs;
      emit = 1;
      word = opcode(op) | (uint32_t)urs << 3 | op_fields(cs, s, e) | m << 18;
    } else {
      const int64_t ol = e - s;
      emit = 1;
      word = 5u | (uint32_t)rs << 3 | (uint32_t)(ol > 63 ? 63 : ol) << 4;
    }
    if (emit) {
      const int64_t w = s / S;
      if (w < nwaves) wcount[w]++;
      out[total++] = word;
    }
    prev = s;
    prev_rs = rs;
    s = e;
  }
  return total;
}
