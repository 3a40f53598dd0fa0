// Test driver for the ASan/UBSan build of csrc/ingest.cpp (host code only):
//   ingest_asan REF PAF READS N_THREADS
// prints "status n_reads n_alignments" and an FNV-1a 64 digest of every output
// array, which tests/test_ingest_sanitized.py compares with the production
// library's output on the same files.
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include "mpc_ingest.h"

static unsigned long long fnv(const void* p, long long n) {
  const unsigned char* b = static_cast<const unsigned char*>(p);
  unsigned long long h = 1469598103934665603ull;
  for (long long i = 0; i < n; ++i) { h ^= b[i]; h *= 1099511628211ull; }
  return h;
}

int main(int argc, char** argv) {
  if (argc != 5) { fprintf(stderr, "usage: %s REF PAF READS N_THREADS\n", argv[0]); return 2; }
  mpc_ingest_out o;
  memset(&o, 0, sizeof o);
  mpc_ingest(argv[1], argv[2], argv[3], atoi(argv[4]), &o);
  printf("%d %lld %lld", o.status, (long long)o.n_reads, (long long)o.n_alignments);
  if (o.status == MPC_INGEST_OK) {
    const long long n = o.n_reads;
    if (!o.cs_off || !o.up_off || !o.down_off) { printf(" null-offsets\n"); return 1; }
    printf(" ref=%016llx", fnv(o.ref, o.ref_len));
    printf(" cs=%016llx", fnv(o.cs, o.cs_off[n]));
    printf(" cs_off=%016llx", fnv(o.cs_off, 8 * (n + 1)));
    printf(" tstart=%016llx", fnv(o.tstart, 8 * n));
    printf(" up=%016llx", fnv(o.up, o.up_off[n]));
    printf(" up_off=%016llx", fnv(o.up_off, 8 * (n + 1)));
    printf(" down=%016llx", fnv(o.down, o.down_off[n]));
    printf(" down_off=%016llx", fnv(o.down_off, 8 * (n + 1)));
    printf(" aligned=%016llx", fnv(o.aligned, 8 * n));
  }
  printf("\n");
  mpc_ingest_free(&o);
  return 0;
}
