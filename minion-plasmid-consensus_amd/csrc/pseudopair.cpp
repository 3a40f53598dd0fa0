// pseudopair.cpp -- native src/pseudopair_reads.py (rule pseudopair_reads,
// Snakefile:211-228) behind include/mpc_ingest.h (host I/O library).
//
// Semantics of /root/reference/src/pseudopair_reads.py:92-140, restated in
// minion-plasmid-consensus_amd/pseudopair_reads.py:
//   per PAF line (file order): split('\t') WITHOUT rstrip; name = field 0;
//   int() of fields 1, 2, 3; strand = field 4 (a 5-field line keeps its '\n'
//   in field 4, so it is not "+"); a name already in the forward or reverse
//   table is deleted from it, else it is added (strand "+" forward, anything
//   else reverse) with aligned length = field 3 - field 2; a later sighting
//   re-adds it at the END of its table's order (dict delete / re-insert).
//   Then lengths < min_align_length are dropped and the i-th forward read is
//   paired with the i-th reverse read ("fwd rev\n") up to the shorter table.
// Lines are split and parsed by all cores; the table pass is sequential (it
// depends on file order).  Inputs this parser does not restate -- integers in a
// form only Python's int() accepts, bytes >= 0x80, '\r' (universal newlines)
// -- are declined (status MPC_INGEST_FALLBACK): the caller uses the Python
// restatement.
#include "host_threads.h"
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <string_view>
#include <thread>
#include <unordered_map>
#include <vector>

#include "mpc_ingest.h"

namespace {

using sv = std::string_view;

struct Rec {
  sv name;
  int64_t length = 0;
  uint8_t plus = 0;
  uint8_t state = 0;  // 0 ok, 1 error (fewer than 5 fields), 2 decline
};

// int() of a field that is a plain optionally-signed run of 1-18 digits; false: not restated here
bool plain_int(sv f, int64_t* out) {
  size_t k = 0;
  bool neg = false;
  if (k < f.size() && (f[k] == '-' || f[k] == '+')) { neg = f[k] == '-'; ++k; }
  if (k == f.size() || f.size() - k > 18) return false;
  int64_t v = 0;
  for (; k < f.size(); ++k) {
    if (f[k] < '0' || f[k] > '9') return false;
    v = v * 10 + (f[k] - '0');
  }
  *out = neg ? -v : v;
  return true;
}

// one line without its '\n' (had_nl: the line ended with one)
Rec parse_line(sv line, bool had_nl) {
  Rec r;
  sv f[5];
  size_t nf = 0, a = 0;
  for (size_t k = 0; k <= line.size() && nf < 5; ++k) {
    if (k == line.size() || line[k] == '\t') {
      f[nf++] = line.substr(a, k - a);
      a = k + 1;
    }
  }
  const bool more = nf == 5 && a <= line.size();  // a sixth field follows field 4
  if (nf < 5) { r.state = 1; return r; }          // f[4] -> IndexError (after the int()s, also exit 1)
  int64_t qlen, qs, qe;
  if (!plain_int(f[1], &qlen) || !plain_int(f[2], &qs) || !plain_int(f[3], &qe)) { r.state = 2; return r; }
  r.name = f[0];
  r.length = qe - qs;
  // field 4 is the line's last field only when no tab follows it: then it keeps the newline
  r.plus = f[4] == "+" && (more || !had_nl);
  return r;
}

}  // namespace

extern "C" {

int mpc_pseudopair(const char* paf_path, int64_t min_align_length, int has_min, const char* out_path, int n_threads,
                   mpc_pseudopair_stats* st) {
  std::memset(st, 0, sizeof(*st));
  auto fail = [&](int status, const std::string& m) {
    st->status = status;
    std::snprintf(st->message, sizeof st->message, "%s", m.c_str());
    return status;
  };
  const int fd = ::open(paf_path, O_RDONLY);
  if (fd < 0) return fail(MPC_INGEST_ERROR, std::string("cannot open ") + paf_path);
  struct stat sb;
  if (fstat(fd, &sb) != 0) { ::close(fd); return fail(MPC_INGEST_ERROR, "stat failed"); }
  const size_t n = (size_t)sb.st_size;
  const char* p = "";
  void* m = nullptr;
  if (n) {
    m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) { ::close(fd); return fail(MPC_INGEST_ERROR, "mmap failed"); }
    p = static_cast<const char*>(m);
  }
  struct Unmap {
    void* m; size_t n; int fd;
    ~Unmap() { if (m) munmap(m, n); ::close(fd); }
  } unmap{m, n, fd};
  const sv text(p, n);
  // line starts
  std::vector<size_t> starts;
  for (size_t k = 0; k < n;) {
    starts.push_back(k);
    const void* nl = std::memchr(p + k, '\n', n - k);
    k = nl ? (size_t)(static_cast<const char*>(nl) - p) + 1 : n;
  }
  const size_t L = starts.size();
  std::vector<Rec> recs(L);
  int nt = n_threads > 0 ? n_threads : mpc_host::host_threads();
  nt = (int)std::max<size_t>(1, std::min<size_t>((size_t)nt, L / 4096 + 1));
  std::vector<uint8_t> odd((size_t)nt, 0);  // bytes the parser declines
  auto work = [&](int t) {
    for (size_t i = L * t / nt; i < L * (t + 1) / nt; ++i) {
      const size_t a = starts[i], b = i + 1 < L ? starts[i + 1] : n;
      const bool nl = b > a && p[b - 1] == '\n';
      const sv line = text.substr(a, b - a - (nl ? 1 : 0));
      for (char c : line)
        if ((unsigned char)c >= 0x80 || c == '\r') { odd[(size_t)t] = 1; return; }
      recs[i] = parse_line(line, nl);
    }
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t) th.emplace_back(work, t);
  for (auto& x : th) x.join();
  for (uint8_t o : odd)
    if (o) return fail(MPC_INGEST_FALLBACK, "non-ASCII byte or carriage return");
  // the tables, in file order (the first failing line ends the script: later lines never matter)
  struct Entry { sv name; int64_t length; uint8_t plus, alive; };
  std::vector<Entry> ent;
  ent.reserve(L);
  std::unordered_map<sv, size_t> live;
  live.reserve(L * 2 + 16);
  for (size_t i = 0; i < L; ++i) {
    const Rec& r = recs[i];
    if (r.state == 2) return fail(MPC_INGEST_FALLBACK, "integer form not restated natively");
    if (r.state == 1) return fail(MPC_INGEST_ERROR, "IndexError: list index out of range (PAF line " + std::to_string(i + 1) + ")");
    auto it = live.find(r.name);
    if (it != live.end()) {
      ent[it->second].alive = 0;
      live.erase(it);
    } else {
      live.emplace(r.name, ent.size());
      ent.push_back({r.name, r.length, r.plus, 1});
    }
  }
  std::vector<const Entry*> fwd, rev;
  for (const Entry& e : ent) {
    if (!e.alive) continue;
    if (e.plus) ++st->n_fwd; else ++st->n_rev;
  }
  if ((st->n_fwd || st->n_rev) && !has_min)
    return fail(MPC_INGEST_ERROR, "TypeError: '<' not supported between instances of 'int' and 'NoneType'");
  for (const Entry& e : ent) {
    if (!e.alive || e.length < min_align_length) continue;
    (e.plus ? fwd : rev).push_back(&e);
  }
  st->n_fwd_kept = (int64_t)fwd.size();
  st->n_rev_kept = (int64_t)rev.size();
  const size_t np = std::min(fwd.size(), rev.size());
  std::string out;
  for (size_t k = 0; k < np; ++k) {
    out.append(fwd[k]->name);
    out += ' ';
    out.append(rev[k]->name);
    out += '\n';
  }
  st->n_pairs = (int64_t)np;
  FILE* f = std::fopen(out_path, "wb");
  if (!f) return fail(MPC_INGEST_ERROR, std::string("cannot open ") + out_path + " for writing");
  const bool ok = std::fwrite(out.data(), 1, out.size(), f) == out.size();
  if (std::fclose(f) != 0 || !ok) return fail(MPC_INGEST_ERROR, "write error");
  st->status = MPC_INGEST_OK;
  return MPC_INGEST_OK;
}

}  // extern "C"
