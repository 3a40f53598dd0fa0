// Seeded synthetic cs-tagged alignment generator (host C++, C-ABI).
//
// Produces, for one plasmid reference, N reads aligned with minimap2-style
// short cs tags, in exactly the packed form the host ingest hands to the
// device path (SURVEY.md §8(d) "Synthetic inputs"):
//   * sample 0 ("sense"):     alignments to ref
//   * sample 1 ("antisense"): the same reads aligned to revcomp(ref)
//     (Snakefile:348-378 revcomp_assembly; Snakefile:406 uses ONE reads file
//     for both strands), obtained by reversing + complementing each op list.
// It can also write the text inputs the reference CLI reads
// (ref FASTA, reads FASTA, PAF with cs:Z:), so the same data drives the
// reference script (golden fixtures), the C oracle and the HIP path.
//
// The generator is test/bench infrastructure, not part of the hot path.
#include "host_threads.h"
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>
#include <algorithm>

namespace {

struct Rng {
  uint64_t s[4];
  static uint64_t splitmix(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
  }
  explicit Rng(uint64_t seed) {
    uint64_t x = seed;
    for (auto& v : s) v = splitmix(x);
  }
  static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
  uint64_t next() {
    uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
    s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
    return r;
  }
  double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }  // [0,1)
  int64_t range(int64_t lo, int64_t hi) {                               // [lo,hi]
    if (hi <= lo) return lo;
    return lo + (int64_t)(next() % (uint64_t)(hi - lo + 1));
  }
  // failures before first success, success prob p
  int64_t geom(double p) {
    if (p <= 0.0) return INT64_MAX / 4;
    if (p >= 1.0) return 0;
    double u = 1.0 - uni();  // (0,1]
    double g = std::floor(std::log(u) / std::log1p(-p));
    if (g > 4e18) return INT64_MAX / 4;
    return (int64_t)g;
  }
};

const char kBases[4] = {'A', 'C', 'G', 'T'};
inline char comp(char c) {
  switch (c) {
    case 'A': return 'T'; case 'C': return 'G'; case 'G': return 'C'; case 'T': return 'A';
    case 'a': return 't'; case 'c': return 'g'; case 'g': return 'c'; case 't': return 'a';
    default: return 'N';
  }
}
inline char lower(char c) { return (c >= 'A' && c <= 'Z') ? (char)(c + 32) : c; }
inline char upper(char c) { return (c >= 'a' && c <= 'z') ? (char)(c - 32) : c; }
std::string revcomp(const std::string& s) {
  std::string r(s.size(), 'N');
  for (size_t i = 0; i < s.size(); ++i) r[s.size() - 1 - i] = comp(s[i]);
  return r;
}

enum OpT : uint8_t { M = 0, S = 1, I = 2, D = 3 };
struct Op { OpT t; int64_t len; std::string b; };  // S: b = {refbase, readbase}

}  // namespace

extern "C" {

typedef struct {
  int64_t n;            // reference length (random ACGT)
  int64_t n_reads;
  double p_sub, p_ins, p_del;
  int32_t ins_min, ins_max, del_min, del_max;
  int32_t flank_min, flank_max;
  double frac_partial;  // reads with start/end uniform inside the ref
  double frac_minus;    // reads on the '-' strand
  uint64_t seed;
  int32_t antisense;    // also produce sample 1 (alignments to revcomp(ref))
  int32_t n_threads;
  // generate only reads [read_begin, read_end) of the n_reads-read set (both 0:
  // all of them).  Every read is keyed by (seed, global index), so the shards of
  // a multi-GPU run are exact slices of the one global read set.
  int64_t read_begin, read_end;
} mpc_synth_params;

struct SynthSample {
  std::string ref;
  std::vector<char> cs;          // "Z:" + body, concatenated
  std::vector<int64_t> cs_off;   // N+1
  std::vector<int64_t> tstart, tend, aligned, nmatch, blen;
  std::vector<char> up, down;    // flanks in this sample's reference orientation
  std::vector<int64_t> up_off, down_off;
  std::vector<char> strand;      // '+' / '-'
};
struct SynthHandle {
  mpc_synth_params p;
  SynthSample s[2];
  std::vector<int64_t> qlen, qs, qe;  // PAF query coords (same for both samples)
};

enum {
  MPC_SYN_REF = 0, MPC_SYN_CS, MPC_SYN_CS_OFF, MPC_SYN_TSTART, MPC_SYN_UP, MPC_SYN_UP_OFF,
  MPC_SYN_DOWN, MPC_SYN_DOWN_OFF, MPC_SYN_ALIGNED, MPC_SYN_STRAND, MPC_SYN_TEND
};

static void gen_read(const mpc_synth_params& p, const std::string& ref, uint64_t ridx,
                     std::vector<Op>& ops, int64_t& ts, int64_t& te, std::string& up,
                     std::string& down, bool& minus, int64_t& nmatch, int64_t& alen) {
  const int64_t n = (int64_t)ref.size();
  Rng rng(p.seed * 0x100000001B3ull ^ (ridx + 1) * 0x9E3779B97F4A7C15ull);
  ops.clear();
  ts = 0; te = n;
  if (rng.uni() < p.frac_partial && n >= 4) {
    int64_t minlen = std::min<int64_t>(20, n);
    for (int tries = 0; tries < 64; ++tries) {
      int64_t a = rng.range(0, n - 1), b = rng.range(0, n);
      if (a > b) std::swap(a, b);
      if (b - a >= minlen) { ts = a; te = b; break; }
    }
  }
  minus = rng.uni() < p.frac_minus;
  const double q = p.p_sub + p.p_del;
  const double pdel_frac = q > 0 ? p.p_del / q : 0.0;
  int64_t j = ts, run = 0;
  nmatch = 0; alen = 0;
  auto flush = [&]() {
    if (run > 0) { ops.push_back({M, run, std::string()}); nmatch += run; alen += run; run = 0; }
  };
  int64_t nsd = ts + rng.geom(q);
  int64_t nins = ts + rng.geom(p.p_ins);
  while (true) {
    // ordering key: sub/del at position x -> 2x ; insertion after position a -> 2a+1
    int64_t ksd = nsd < te ? 2 * nsd : INT64_MAX;
    int64_t kin = nins < te ? 2 * nins + 1 : INT64_MAX;
    if (ksd == INT64_MAX && kin == INT64_MAX) break;
    if (ksd < kin) {
      int64_t x = nsd;
      run += x - j; j = x;
      if (rng.uni() < pdel_frac) {
        int64_t L = rng.range(p.del_min, p.del_max);
        if (L >= 1 && x > ts && x + L < te) {
          flush();
          ops.push_back({D, L, ref.substr((size_t)x, (size_t)L)});
          j = x + L;
        } else {
          run += 1; j = x + 1;
        }
      } else {
        char rb = ref[(size_t)x];
        char yb = rb;
        while (yb == rb) yb = kBases[rng.next() & 3];
        flush();
        ops.push_back({S, 1, std::string{rb, yb}});
        alen += 1;
        j = x + 1;
      }
      nsd = j + rng.geom(q);
      if (nins < j - 1) nins = j - 1 + rng.geom(p.p_ins);
    } else {
      int64_t a = nins;
      run += (a + 1) - j; j = a + 1;
      if (a >= ts && a + 1 < te) {
        int64_t L = rng.range(p.ins_min, p.ins_max);
        if (L >= 1) {
          std::string b((size_t)L, 'A');
          for (auto& c : b) c = kBases[rng.next() & 3];
          flush();
          ops.push_back({I, L, b});
          alen += L;
        }
      }
      nins = a + 1 + rng.geom(p.p_ins);
    }
  }
  run += te - j;
  flush();
  int64_t ul = rng.range(p.flank_min, p.flank_max), dl = rng.range(p.flank_min, p.flank_max);
  up.assign((size_t)ul, 'A');
  down.assign((size_t)dl, 'A');
  for (auto& c : up) c = kBases[rng.next() & 3];
  for (auto& c : down) c = kBases[rng.next() & 3];
}

static void emit_cs(const std::vector<Op>& ops, bool reverse, std::string& cs) {
  cs.assign("Z:");
  char buf[32];
  auto one = [&](const Op& o) {
    switch (o.t) {
      case M: snprintf(buf, sizeof buf, ":%lld", (long long)o.len); cs += buf; break;
      case S:
        cs += '*';
        if (!reverse) { cs += lower(o.b[0]); cs += lower(o.b[1]); }
        else { cs += lower(comp(o.b[0])); cs += lower(comp(o.b[1])); }
        break;
      case I: case D: {
        cs += (o.t == I) ? '+' : '-';
        std::string s = reverse ? revcomp(o.b) : o.b;
        for (char c : s) cs += lower(c);
        break;
      }
    }
  };
  if (!reverse) for (const auto& o : ops) one(o);
  else for (auto it = ops.rbegin(); it != ops.rend(); ++it) one(*it);
}

void* mpc_synth_new(const mpc_synth_params* pp) {
  auto* h = new SynthHandle();
  h->p = *pp;
  const auto& p = h->p;
  Rng rr(p.seed ^ 0xC0FFEEull);
  std::string ref((size_t)p.n, 'A');
  for (auto& c : ref) c = kBases[rr.next() & 3];
  const int ns = p.antisense ? 2 : 1;
  h->s[0].ref = ref;
  if (ns == 2) h->s[1].ref = revcomp(ref);
  int64_t R0 = p.read_begin, R1 = p.read_end;
  if (R0 == 0 && R1 == 0) R1 = p.n_reads;
  R0 = std::max<int64_t>(0, std::min<int64_t>(R0, p.n_reads));
  R1 = std::max<int64_t>(R0, std::min<int64_t>(R1, p.n_reads));
  h->p.read_begin = R0;
  h->p.read_end = R1;
  const int64_t N = R1 - R0;
  int nt = p.n_threads > 0 ? p.n_threads : mpc_host::host_threads();
  nt = std::min(nt, 16);  // the GPU box's CPU share
  nt = (int)std::min<int64_t>(nt, std::max<int64_t>(1, N / 256));
  struct Part {
    std::vector<char> cs[2], up[2], down[2];
    std::vector<int64_t> cs_len[2], up_len[2], down_len[2], ts[2], te[2], al, nm, bl;
    std::vector<char> strand[2];
    std::vector<int64_t> qlen, qs, qe;
  };
  std::vector<Part> parts((size_t)nt);
  auto work = [&](int t) {
    Part& P = parts[(size_t)t];
    int64_t r0 = N * t / nt, r1 = N * (t + 1) / nt;
    std::vector<Op> ops;
    std::string up, down, cs;
    for (int64_t r = r0; r < r1; ++r) {
      int64_t ts, te, nm, al;
      bool minus;
      gen_read(p, ref, (uint64_t)(R0 + r), ops, ts, te, up, down, minus, nm, al);
      int64_t blen = 0;
      for (auto& o : ops) blen += o.len;
      P.al.push_back(al); P.nm.push_back(nm); P.bl.push_back(blen);
      int64_t qlen = (int64_t)up.size() + al + (int64_t)down.size();
      P.qlen.push_back(qlen);
      // PAF query coordinates on the read as written to the FASTA
      if (!minus) { P.qs.push_back((int64_t)up.size()); P.qe.push_back((int64_t)up.size() + al); }
      else { P.qs.push_back((int64_t)down.size()); P.qe.push_back((int64_t)down.size() + al); }
      for (int s = 0; s < ns; ++s) {
        bool rev = (s == 1);
        emit_cs(ops, rev, cs);
        P.cs[s].insert(P.cs[s].end(), cs.begin(), cs.end());
        P.cs_len[s].push_back((int64_t)cs.size());
        std::string u = rev ? revcomp(down) : up;
        std::string d = rev ? revcomp(up) : down;
        P.up[s].insert(P.up[s].end(), u.begin(), u.end());
        P.down[s].insert(P.down[s].end(), d.begin(), d.end());
        P.up_len[s].push_back((int64_t)u.size());
        P.down_len[s].push_back((int64_t)d.size());
        P.ts[s].push_back(rev ? p.n - te : ts);
        P.te[s].push_back(rev ? p.n - ts : te);
        bool m = rev ? !minus : minus;
        P.strand[s].push_back(m ? '-' : '+');
      }
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
  for (auto& x : th) x.join();
  for (int s = 0; s < ns; ++s) {
    SynthSample& S_ = h->s[s];
    S_.cs_off.assign(1, 0); S_.up_off.assign(1, 0); S_.down_off.assign(1, 0);
    for (auto& P : parts) {
      S_.cs.insert(S_.cs.end(), P.cs[s].begin(), P.cs[s].end());
      S_.up.insert(S_.up.end(), P.up[s].begin(), P.up[s].end());
      S_.down.insert(S_.down.end(), P.down[s].begin(), P.down[s].end());
      for (auto l : P.cs_len[s]) S_.cs_off.push_back(S_.cs_off.back() + l);
      for (auto l : P.up_len[s]) S_.up_off.push_back(S_.up_off.back() + l);
      for (auto l : P.down_len[s]) S_.down_off.push_back(S_.down_off.back() + l);
      S_.tstart.insert(S_.tstart.end(), P.ts[s].begin(), P.ts[s].end());
      S_.tend.insert(S_.tend.end(), P.te[s].begin(), P.te[s].end());
      S_.aligned.insert(S_.aligned.end(), P.al.begin(), P.al.end());
      S_.nmatch.insert(S_.nmatch.end(), P.nm.begin(), P.nm.end());
      S_.blen.insert(S_.blen.end(), P.bl.begin(), P.bl.end());
      S_.strand.insert(S_.strand.end(), P.strand[s].begin(), P.strand[s].end());
      if (s == 0) {
        h->qlen.insert(h->qlen.end(), P.qlen.begin(), P.qlen.end());
        h->qs.insert(h->qs.end(), P.qs.begin(), P.qs.end());
        h->qe.insert(h->qe.end(), P.qe.begin(), P.qe.end());
      }
    }
  }
  return h;
}

void mpc_synth_free(void* hv) { delete (SynthHandle*)hv; }

static const void* field(SynthHandle* h, int what, int s, int64_t* count, int* elem) {
  SynthSample& S_ = h->s[s];
  switch (what) {
    case MPC_SYN_REF: *count = (int64_t)S_.ref.size(); *elem = 1; return S_.ref.data();
    case MPC_SYN_CS: *count = (int64_t)S_.cs.size(); *elem = 1; return S_.cs.data();
    case MPC_SYN_CS_OFF: *count = (int64_t)S_.cs_off.size(); *elem = 8; return S_.cs_off.data();
    case MPC_SYN_TSTART: *count = (int64_t)S_.tstart.size(); *elem = 8; return S_.tstart.data();
    case MPC_SYN_UP: *count = (int64_t)S_.up.size(); *elem = 1; return S_.up.data();
    case MPC_SYN_UP_OFF: *count = (int64_t)S_.up_off.size(); *elem = 8; return S_.up_off.data();
    case MPC_SYN_DOWN: *count = (int64_t)S_.down.size(); *elem = 1; return S_.down.data();
    case MPC_SYN_DOWN_OFF: *count = (int64_t)S_.down_off.size(); *elem = 8; return S_.down_off.data();
    case MPC_SYN_ALIGNED: *count = (int64_t)S_.aligned.size(); *elem = 8; return S_.aligned.data();
    case MPC_SYN_STRAND: *count = (int64_t)S_.strand.size(); *elem = 1; return S_.strand.data();
    case MPC_SYN_TEND: *count = (int64_t)S_.tend.size(); *elem = 8; return S_.tend.data();
  }
  *count = -1; *elem = 0; return nullptr;
}

int64_t mpc_synth_size(void* hv, int what, int s) {
  int64_t c; int e;
  field((SynthHandle*)hv, what, s, &c, &e);
  return c < 0 ? -1 : c * e;
}

int mpc_synth_copy(void* hv, int what, int s, void* dst) {
  int64_t c; int e;
  const void* src = field((SynthHandle*)hv, what, s, &c, &e);
  if (!src && c < 0) return -1;
  if (c > 0) memcpy(dst, src, (size_t)(c * e));
  return 0;
}

// Rebuild the aligned query bases (reference orientation of sample 0) from a cs body.
static void query_from_cs(const std::string& ref, int64_t ts, const char* cs, int64_t len, std::string& out) {
  out.clear();
  int64_t i = ts, k = 2;  // skip "Z:"
  while (k < len) {
    char op = cs[k++];
    int64_t s = k;
    while (k < len && !strchr(":*+-Z", cs[k])) ++k;
    if (op == ':') {
      int64_t L = 0;
      for (int64_t q = s; q < k; ++q) L = L * 10 + (cs[q] - '0');
      out.append(ref, (size_t)i, (size_t)L);
      i += L;
    } else if (op == '*') { out += upper(cs[k - 1]); i += 1; }
    else if (op == '+') { for (int64_t q = s; q < k; ++q) out += upper(cs[q]); }
    else if (op == '-') { i += k - s; }
  }
}

static void write_wrapped(FILE* f, const std::string& s, size_t w) {
  for (size_t i = 0; i < s.size(); i += w) {
    fwrite(s.data() + i, 1, std::min(w, s.size() - i), f);
    fputc('\n', f);
  }
  if (s.empty()) fputc('\n', f);
}

// Write reference-CLI inputs. Any path may be NULL to skip it.
int mpc_synth_write_files(void* hv, const char* ref_fa, const char* reads_fa, const char* paf0,
                          const char* ref_as_fa, const char* paf1) {
  auto* h = (SynthHandle*)hv;
  const auto& p = h->p;
  const int64_t N = p.read_end - p.read_begin, R0 = p.read_begin;
  if (ref_fa) {
    FILE* f = fopen(ref_fa, "w"); if (!f) return -1;
    fputs(">tig00000001 len=", f); fprintf(f, "%lld\n", (long long)p.n);
    write_wrapped(f, h->s[0].ref, 60); fclose(f);
  }
  if (ref_as_fa && p.antisense) {
    FILE* f = fopen(ref_as_fa, "w"); if (!f) return -1;
    fputs(">tig00000001_revcomp\n", f);
    write_wrapped(f, h->s[1].ref, 60); fclose(f);
  }
  if (reads_fa) {
    FILE* f = fopen(reads_fa, "w"); if (!f) return -1;
    const SynthSample& S0 = h->s[0];
    std::string q, full;
    for (int64_t r = 0; r < N; ++r) {
      int64_t a = S0.cs_off[(size_t)r], b = S0.cs_off[(size_t)r + 1];
      query_from_cs(S0.ref, S0.tstart[(size_t)r], S0.cs.data() + a, b - a, q);
      full.assign(S0.up.data() + S0.up_off[(size_t)r], (size_t)(S0.up_off[(size_t)r + 1] - S0.up_off[(size_t)r]));
      full += q;
      full.append(S0.down.data() + S0.down_off[(size_t)r], (size_t)(S0.down_off[(size_t)r + 1] - S0.down_off[(size_t)r]));
      if (S0.strand[(size_t)r] == '-') full = revcomp(full);
      fprintf(f, ">read_%lld\n", (long long)(R0 + r));
      write_wrapped(f, full, 80);
    }
    fclose(f);
  }
  const char* pafs[2] = {paf0, paf1};
  for (int s = 0; s < (p.antisense ? 2 : 1); ++s) {
    if (!pafs[s]) continue;
    FILE* f = fopen(pafs[s], "w"); if (!f) return -1;
    const SynthSample& S_ = h->s[s];
    for (int64_t r = 0; r < N; ++r) {
      size_t ri = (size_t)r;
      fprintf(f, "read_%lld\t%lld\t%lld\t%lld\t%c\t%s\t%lld\t%lld\t%lld\t%lld\t%lld\t60\ttp:A:P\tcs:",
              (long long)(R0 + r), (long long)h->qlen[ri], (long long)h->qs[ri], (long long)h->qe[ri],
              S_.strand[ri], s ? "tig00000001_revcomp" : "tig00000001", (long long)p.n,
              (long long)S_.tstart[ri], (long long)S_.tend[ri], (long long)S_.nmatch[ri],
              (long long)S_.blen[ri]);
      fwrite(S_.cs.data() + S_.cs_off[ri], 1, (size_t)(S_.cs_off[ri + 1] - S_.cs_off[ri]), f);
      fputc('\n', f);
    }
    fclose(f);
  }
  return 0;
}

}  // extern "C"
