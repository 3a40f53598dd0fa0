/*
 * mpc_oracle.c -- CPU restatement of the reference pileup + consensus.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load this library; the product path
 * (minion-plasmid-consensus_amd/) never links, imports or calls it.
 *
 * It restates, step for step, the algorithm of the reference script
 * /root/reference/src/mapped_paf_read_parser.py (v5.1):
 *   processBaseString_leftIndel   :37-62   -> left_indel()   (front insertion, right-justified)
 *   processBaseString_rightIndel  :64-72   -> right_indel()  (append, left-justified)
 *   processOperation              :74-104  -> process_op()
 *   Step 4 cs tokenizer           :285-323 -> oracle_pileup()
 *   Step 5 max depth              :332-341
 *   Step 6 consensus              :348-439 -> oracle_consensus()
 * on the packed per-read inputs the reference builds in Steps 1-3
 * (refseq, tstart, cs text after "cs:", upstream/downstream flanks).
 * Slots are kept as a per-position array with memmove front insertion,
 * exactly like the Python list.insert(0, ...) it mirrors.
 *
 * Pinned against the reference itself: tests/golden/ holds outputs of the
 * reference script on seeded inputs (scripts/make_golden.py) and
 * tests/test_oracle_golden.py checks this file against every one of them.
 *
 * Error kinds map to the reference's exceptions (all exit status 1):
 *   ORC_E_KEY    KeyError   (non-ACGT base written; :61, :71)
 *   ORC_E_INDEX  IndexError (position past the reference; :57/:69/:79, '*' with empty operand :96)
 *   ORC_E_VALUE  ValueError (int() of a ':' operand; :77)
 *   ORC_E_OP     sys.exit("Unknown operator") (:100-102)
 * Indices follow Python's list semantics exactly, negative wrap included
 * (obs_index): a negative target start (never written by minimap2) reaches
 * refarr / obsarr at len + index, like the reference (:222, :300-303, :57-61,
 * :69, :79, :87, :96), pinned by tests/golden/n_neg_*.  The HIP path
 * implements all of it on one shard, including the strings the wrap writes
 * into odd positions (K_woprep .. K_worows, include/mpc.h).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

enum { ORC_OK = 0, ORC_E_KEY = 1, ORC_E_INDEX = 2, ORC_E_VALUE = 3, ORC_E_OP = 4, ORC_E_NOMEM = 5 };

typedef struct { int64_t c[4]; } Slot; /* dict order of the reference: A, T, C, G (:59, :70) */
typedef struct { Slot* s; int32_t len, cap; } Pos;

typedef struct {
  int64_t n_calls;
  char* base;      /* consensus base after the GTF test (:421-423) */
  char* chrom1;    /* pre-GTF top base (:417) */
  char* chrom2;    /* second base (:418) */
  int64_t* count;
  int64_t* count2;
  int64_t* total;  /* sum over the slot, denominator of the accuracy (:431) */
  int64_t* xpos;   /* obsarr index x of the slot (debug) */
  int64_t* slot;   /* base_pos within obsarr[x] (debug) */
  int64_t max_depth;
  int err;
  int64_t err_read;
} orc_out;

static int code_of(char b) {
  switch (b) { case 'A': return 0; case 'T': return 1; case 'C': return 2; case 'G': return 3; }
  return -1;
}
static const char kName[4] = {'A', 'T', 'C', 'G'};
static char upc(char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 32) : c; }

static int grow(Pos* p) {
  if (p->len < p->cap) return 0;
  int32_t nc = p->cap ? p->cap * 2 : 4;
  Slot* ns = (Slot*)realloc(p->s, sizeof(Slot) * (size_t)nc);
  if (!ns) return ORC_E_NOMEM;
  p->s = ns; p->cap = nc;
  return 0;
}

/* Python list index: x in [-P, P) -> x mod P, else -1 (IndexError) */
static int64_t obs_index(int64_t x, int64_t P) {
  if (x < 0) x += P;
  return (x < 0 || x >= P) ? -1 : x;
}

/* processBaseString_leftIndel (:37-62) */
static int left_indel(Pos* obs, int64_t P, int64_t x0, const char* str, int64_t L, int upper) {
  const int64_t x = obs_index(x0, P);
  for (int64_t bi = 0; bi < L; ++bi) {
    if (x < 0) return ORC_E_INDEX;
    char b = str[L - bi - 1];
    if (upper) b = upc(b);
    Pos* p = &obs[x];
    if (p->len <= bi) { /* obsarr[i].insert(0, {...}) */
      if (grow(p)) return ORC_E_NOMEM;
      memmove(p->s + 1, p->s, sizeof(Slot) * (size_t)p->len);
      memset(&p->s[0], 0, sizeof(Slot));
      p->len++;
    }
    int k = code_of(b);
    if (k < 0) return ORC_E_KEY;
    p->s[p->len - 1 - bi].c[k] += 1; /* obsarr[i][-(1+bi)][b] += 1 */
  }
  return 0;
}

/* processBaseString_rightIndel (:64-72) */
static int right_indel(Pos* obs, int64_t P, int64_t x0, const char* str, int64_t L) {
  const int64_t x = obs_index(x0, P);
  for (int64_t bi = 0; bi < L; ++bi) {
    if (x < 0) return ORC_E_INDEX;
    char b = str[bi];
    Pos* p = &obs[x];
    if (p->len <= bi) {
      if (grow(p)) return ORC_E_NOMEM;
      memset(&p->s[p->len], 0, sizeof(Slot));
      p->len++;
    }
    int k = code_of(b);
    if (k < 0) return ORC_E_KEY;
    p->s[bi].c[k] += 1;
  }
  return 0;
}

static int is_pyspace(char c) {
  return c == ' ' || c == '\t' || c == '\n' || c == '\r' || c == '\x0b' || c == '\x0c' ||
         (c >= '\x1c' && c <= '\x1f');
}

/* Python int(str) in base 10 restricted to ASCII: strip, optional sign, digits with
 * single '_' separators.  Saturates at 2^62 (the caller hits IndexError long before). */
static int py_int(const char* s, int64_t len, int64_t* out) {
  int64_t a = 0, b = len;
  while (a < b && is_pyspace(s[a])) ++a;
  while (b > a && is_pyspace(s[b - 1])) --b;
  int neg = 0;
  if (a < b && (s[a] == '+' || s[a] == '-')) { neg = s[a] == '-'; ++a; }
  if (a >= b) return ORC_E_VALUE;
  int64_t v = 0;
  int prev_digit = 0;
  for (int64_t k = a; k < b; ++k) {
    char c = s[k];
    if (c >= '0' && c <= '9') {
      if (v < ((int64_t)1 << 62)) v = v * 10 + (c - '0');
      prev_digit = 1;
    } else if (c == '_' && prev_digit && k + 1 < b && s[k + 1] >= '0' && s[k + 1] <= '9') {
      prev_digit = 0;
    } else {
      return ORC_E_VALUE;
    }
  }
  if (!prev_digit) return ORC_E_VALUE;
  *out = neg ? -v : v;
  return 0;
}

/* processOperation (:74-104); i is the reference coordinate, updated in place */
static int process_op(Pos* obs, int64_t P, const char* ref, int64_t* i, char op,
                      const char* operand, int64_t olen) {
  if (op == ':') {
    int64_t v;
    int e = py_int(operand, olen, &v);
    if (e) return e;
    for (int64_t x = 0; x < v; ++x) {
      /* refarr[(2*i)+1]: an odd index holds ref[i], an even one (reached by a
       * wrapped negative index) holds '' */
      const int64_t ri = obs_index(2 * (*i) + 1, P);
      if (ri < 0) return ORC_E_INDEX;
      if (ri & 1) {
        e = left_indel(obs, P, ri, ref + (ri - 1) / 2, 1, 0);
        if (e) return e;
      }
      *i += 1;
    }
  } else if (op == '+') {
    int e = left_indel(obs, P, 2 * (*i), operand, olen, 1);
    if (e) return e;
  } else if (op == '-') {
    *i += olen;
  } else if (op == '*') {
    if (olen == 0) return ORC_E_INDEX; /* operand[-1] */
    int e = left_indel(obs, P, 2 * (*i) + 1, operand + olen - 1, 1, 1);
    if (e) return e;
    *i += 1;
  } else if (op == 'Z') {
  } else {
    return ORC_E_OP;
  }
  return 0;
}

static int is_special(char c) { return c == ':' || c == 'Z' || c == '+' || c == '-' || c == '*'; }

/* Step 4 (:285-323) for all reads. */
static int oracle_pileup(Pos* obs, int64_t P, const char* ref, int64_t nreads,
                         const char* cs, const int64_t* cs_off, const int64_t* tstart,
                         const char* up, const int64_t* up_off, const char* down,
                         const int64_t* down_off, int64_t* err_read) {
  for (int64_t r = 0; r < nreads; ++r) {
    int64_t i = tstart[r];
    *err_read = r;
    int e = left_indel(obs, P, 2 * i, up + up_off[r], up_off[r + 1] - up_off[r], 0);
    if (e) return e;
    const char* c = cs + cs_off[r];
    int64_t len = cs_off[r + 1] - cs_off[r];
    char op = 0; /* "" */
    int64_t ostart = 0, olen = 0;
    for (int64_t k = 0; k < len; ++k) {
      if (is_special(c[k])) {
        if (olen != 0) {
          e = process_op(obs, P, ref, &i, op, c + ostart, olen);
          if (e) return e;
        }
        op = c[k];
        ostart = k + 1;
        olen = 0;
      } else {
        olen += 1;
      }
    }
    e = process_op(obs, P, ref, &i, op, c + ostart, olen);
    if (e) return e;
    e = right_indel(obs, P, 2 * i, down + down_off[r], down_off[r + 1] - down_off[r]);
    if (e) return e;
  }
  return 0;
}

static int push_call(orc_out* o, int64_t* cap, char base, char c1, char c2, int64_t cnt,
                     int64_t cnt2, int64_t tot, int64_t x, int64_t slot) {
  if (o->n_calls == *cap) {
    int64_t nc = *cap ? *cap * 2 : 1024;
#define RE(f, T) { T* t = (T*)realloc(o->f, sizeof(T) * (size_t)nc); if (!t) return ORC_E_NOMEM; o->f = t; }
    RE(base, char) RE(chrom1, char) RE(chrom2, char) RE(count, int64_t) RE(count2, int64_t)
    RE(total, int64_t) RE(xpos, int64_t) RE(slot, int64_t)
#undef RE
    *cap = nc;
  }
  int64_t k = o->n_calls++;
  o->base[k] = base; o->chrom1[k] = c1; o->chrom2[k] = c2;
  o->count[k] = cnt; o->count2[k] = cnt2; o->total[k] = tot;
  o->xpos[k] = x; o->slot[k] = slot;
  return 0;
}

/* Steps 5-6 (:332-439). */
static int oracle_consensus(Pos* obs, int64_t P, double mdf, double gtf, orc_out* o) {
  int64_t max_depth = 0;
  for (int64_t x = 0; x < P; ++x) {
    if (obs[x].len > 0) {
      int64_t s = 0;
      for (int k = 0; k < 4; ++k) s += obs[x].s[0].c[k];
      if (s > max_depth) max_depth = s;
    }
  }
  o->max_depth = max_depth;
  double thr = (double)max_depth * mdf;
  int64_t cap = 0;
  for (int64_t x = 0; x < P; ++x) {
    for (int32_t bp = 0; bp < obs[x].len; ++bp) {
      const int64_t* c = obs[x].s[bp].c;
      /* list_of_tuples in dict order (v > 0), then sorted(key=count)[::-1] (:371-374):
       * a stable ascending sort reversed = descending count, ties in REVERSE dict order. */
      int idx[4], m = 0;
      for (int k = 0; k < 4; ++k) if (c[k] > 0) idx[m++] = k;
      for (int a = 1; a < m; ++a) { /* stable insertion sort ascending */
        int t = idx[a], b = a - 1;
        while (b >= 0 && c[idx[b]] > c[t]) { idx[b + 1] = idx[b]; --b; }
        idx[b + 1] = t;
      }
      for (int a = 0; a < m / 2; ++a) { int t = idx[a]; idx[a] = idx[m - 1 - a]; idx[m - 1 - a] = t; }
      char base, base2;
      int64_t count, count2, total = 0;
      for (int a = 0; a < m; ++a) total += c[idx[a]];
      if (m == 0) { base = 'X'; count = 0; }
      else if (m == 1) { base = kName[idx[0]]; count = c[idx[0]]; }
      else if (c[idx[0]] > c[idx[1]]) { base = kName[idx[0]]; count = c[idx[0]]; }
      else {
        base = 'N'; count = 0;
        for (int a = 0; a < m; ++a) if (c[idx[a]] == c[idx[0]]) count += c[idx[a]];
      }
      if (m <= 1) { base2 = 'X'; count2 = 0; }
      else if (m == 2) { base2 = kName[idx[1]]; count2 = c[idx[1]]; }
      else if (c[idx[1]] > c[idx[2]]) { base2 = kName[idx[1]]; count2 = c[idx[1]]; }
      else {
        base2 = 'N'; count2 = 0;
        for (int a = 0; a < m; ++a) if (c[idx[a]] == c[idx[1]]) count2 += c[idx[a]];
      }
      char bc = base, bc2 = base2;
      if ((double)count < gtf * (double)count2) base = 'N';
      if ((double)count > thr) {
        int e = push_call(o, &cap, base, bc, bc2, count, count2, total, x, bp);
        if (e) return e;
      }
    }
  }
  return 0;
}

int mpc_oracle_run(const char* ref, int64_t n, int64_t nreads, const char* cs, const int64_t* cs_off,
                   const int64_t* tstart, const char* up, const int64_t* up_off, const char* down,
                   const int64_t* down_off, double mdf, double gtf, orc_out* out) {
  memset(out, 0, sizeof(*out));
  out->err_read = -1;
  int64_t P = 2 * n + 1;
  Pos* obs = (Pos*)calloc((size_t)P, sizeof(Pos));
  if (!obs) { out->err = ORC_E_NOMEM; return out->err; }
  int64_t er = -1;
  int e = oracle_pileup(obs, P, ref, nreads, cs, cs_off, tstart, up, up_off, down, down_off, &er);
  if (e) { out->err = e; out->err_read = er; }
  else { e = oracle_consensus(obs, P, mdf, gtf, out); out->err = e; }
  for (int64_t x = 0; x < P; ++x) free(obs[x].s);
  free(obs);
  return out->err;
}

void mpc_oracle_free(orc_out* o) {
  free(o->base); free(o->chrom1); free(o->chrom2); free(o->count); free(o->count2);
  free(o->total); free(o->xpos); free(o->slot);
  memset(o, 0, sizeof(*o));
}
