// writers.cpp -- native Step 7 writers of /root/reference/src/mapped_paf_read_parser.py
// (:446-463) behind include/mpc_ingest.h (host I/O library libmpc_ingest.so).
//
// Input: one sample's calls exactly as the device returns them (uint32 x4 per
// emitted slot: base | chrom1 << 8 | chrom2 << 16, count, count2, total).
//   consensus   ">consensus\n" + bases + "\n"                          (:447-449)
//   chromat     "pos\tbase\tcount\n", then per call two lines: the pre-GTF
//               top base and the second base, pos = 1-based call index  (:453-457)
//   accuracies  "pos\taccuracy\n", then per call str(100 * (count / total)):
//               f64 division then one f64 multiply, printed like Python's
//               float repr (shortest round-trip digits, fixed notation for
//               decimal exponents in (-4, 16], else e-notation)          (:431, :460-463)
// The calls are formatted by all cores in chunks and written in order.  Only the
// formatting happens before any file is opened; the three files are then opened
// and written one after the other, as the reference does (:447, :453, :460), so
// an open/write failure on a later file leaves the earlier ones written, exactly
// like the reference (Snakemake removes the outputs of a failed job).
#include "host_threads.h"
#include <charconv>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "mpc_ingest.h"

namespace {

// Python's repr(float) (float_repr_style 'short', CPython format_float_short
// with mode 'r' and Py_DTSF_ADD_DOT_0): returns the length written to out (<= 32).
int py_repr(double x, char* out) {
  char* o = out;
  if (std::isnan(x)) { std::memcpy(o, "nan", 3); return 3; }
  if (std::signbit(x)) { *o++ = '-'; x = -x; }
  if (std::isinf(x)) { std::memcpy(o, "inf", 3); return (int)(o - out) + 3; }
  char sci[40];
  const auto r = std::to_chars(sci, sci + sizeof sci, x, std::chars_format::scientific);  // shortest round trip
  const char* e = static_cast<const char*>(std::memchr(sci, 'e', (size_t)(r.ptr - sci)));
  char digits[24];
  int nd = 0;
  for (const char* c = sci; c < e; ++c)
    if (*c != '.') digits[nd++] = *c;
  int exp10 = 0;
  std::from_chars(e + 1 + (e[1] == '+' ? 1 : 0), r.ptr, exp10);
  const int decpt = exp10 + 1;  // the decimal point sits after decpt digits
  if (decpt > -4 && decpt <= 16) {
    if (decpt <= 0) {
      *o++ = '0'; *o++ = '.';
      for (int k = 0; k < -decpt; ++k) *o++ = '0';
      for (int k = 0; k < nd; ++k) *o++ = digits[k];
    } else if (decpt >= nd) {
      for (int k = 0; k < nd; ++k) *o++ = digits[k];
      for (int k = nd; k < decpt; ++k) *o++ = '0';
      *o++ = '.'; *o++ = '0';
    } else {
      for (int k = 0; k < decpt; ++k) *o++ = digits[k];
      *o++ = '.';
      for (int k = decpt; k < nd; ++k) *o++ = digits[k];
    }
  } else {
    *o++ = digits[0];
    if (nd > 1) {
      *o++ = '.';
      for (int k = 1; k < nd; ++k) *o++ = digits[k];
    }
    *o++ = 'e';
    const int ex = decpt - 1;
    *o++ = ex < 0 ? '-' : '+';
    const int ax = ex < 0 ? -ex : ex;
    if (ax < 10) *o++ = '0';
    o = std::to_chars(o, o + 8, ax).ptr;
  }
  return (int)(o - out);
}

inline char* put_u64(char* o, uint64_t v) { return std::to_chars(o, o + 24, v).ptr; }

// chromat and accuracies text of calls [a, b)
void format_range(const uint32_t* calls, int64_t a, int64_t b, std::string* chrom, std::string* acc) {
  chrom->resize((size_t)(b - a) * 2 * 36);
  acc->resize((size_t)(b - a) * 48);
  char* c = chrom->data();
  char* q = acc->data();
  for (int64_t k = a; k < b; ++k) {
    const uint32_t* v = calls + 4 * k;
    const uint64_t pos = (uint64_t)k + 1;
    c = put_u64(c, pos); *c++ = '\t'; *c++ = (char)((v[0] >> 8) & 0xffu); *c++ = '\t'; c = put_u64(c, v[1]); *c++ = '\n';
    c = put_u64(c, pos); *c++ = '\t'; *c++ = (char)((v[0] >> 16) & 0xffu); *c++ = '\t'; c = put_u64(c, v[2]); *c++ = '\n';
    q = put_u64(q, pos); *q++ = '\t';
    q += py_repr(100.0 * ((double)v[1] / (double)v[3]), q);  // :431 100 * (count / total)
    *q++ = '\n';
  }
  chrom->resize((size_t)(c - chrom->data()));
  acc->resize((size_t)(q - acc->data()));
}

bool write_all(const char* path, const std::vector<const std::string*>& parts, char* msg, int msg_len) {
  FILE* f = std::fopen(path, "wb");
  if (!f) { std::snprintf(msg, (size_t)msg_len, "cannot open %s for writing", path); return false; }
  bool ok = true;
  for (const std::string* s : parts) ok &= std::fwrite(s->data(), 1, s->size(), f) == s->size();
  ok &= std::fclose(f) == 0;
  if (!ok) std::snprintf(msg, (size_t)msg_len, "write error on %s", path);
  return ok;
}

}  // namespace

extern "C" {

int mpc_py_float_repr(double x, char* out, int out_len) {
  char buf[40];
  const int n = py_repr(x, buf);
  if (n + 1 > out_len) return -1;
  std::memcpy(out, buf, (size_t)n);
  out[n] = 0;
  return n;
}

int mpc_write_calls(const uint32_t* calls, int64_t n_calls, const char* consensus_path, const char* chromat_path,
                    const char* accuracies_path, int n_threads, char* msg, int msg_len) {
  if (n_calls < 0 || (n_calls > 0 && !calls)) { std::snprintf(msg, (size_t)msg_len, "bad arguments"); return -1; }
  int nt = n_threads > 0 ? n_threads : mpc_host::host_threads();
  nt = (int)std::min<int64_t>(nt, std::max<int64_t>(1, n_calls / 8192));
  std::string cons;
  cons.reserve((size_t)n_calls + 16);
  cons += ">consensus\n";
  for (int64_t k = 0; k < n_calls; ++k) cons += (char)(calls[4 * k] & 0xffu);
  cons += '\n';
  std::vector<std::string> chrom((size_t)nt), acc((size_t)nt);
  std::vector<std::thread> th;
  for (int t = 0; t < nt; ++t)
    th.emplace_back(format_range, calls, n_calls * t / nt, n_calls * (t + 1) / nt, &chrom[(size_t)t], &acc[(size_t)t]);
  for (auto& x : th) x.join();
  static const std::string h_chrom = "pos\tbase\tcount\n", h_acc = "pos\taccuracy\n";
  std::vector<const std::string*> pc{&h_chrom}, pa{&h_acc};
  for (int t = 0; t < nt; ++t) { pc.push_back(&chrom[(size_t)t]); pa.push_back(&acc[(size_t)t]); }
  if (!write_all(consensus_path, {&cons}, msg, msg_len)) return -1;
  if (!write_all(chromat_path, pc, msg, msg_len)) return -1;
  if (!write_all(accuracies_path, pa, msg, msg_len)) return -1;
  return 0;
}

}  // extern "C"
