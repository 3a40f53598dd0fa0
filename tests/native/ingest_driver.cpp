// Test driver for the ASan/UBSan build of the host I/O library (csrc/ingest.cpp,
// writers.cpp, pseudopair.cpp; host code only):
//   ingest_asan REF PAF READS N_THREADS   -> "status n_reads n_alignments" + FNV-1a 64
//                                            digests of every output array
//   ingest_asan pseudopair PAF MIN OUT    -> "status n_fwd n_rev n_fwd_kept n_rev_kept n_pairs"
//   ingest_asan writecalls N SEED C CH ACC -> writes N pseudo-random calls
// tests/test_ingest_sanitized.py compares these with the production library.
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

static int pseudopair_mode(char** argv) {
  mpc_pseudopair_stats st;
  mpc_pseudopair(argv[2], atoll(argv[3]), 1, argv[4], 3, &st);
  printf("%d %lld %lld %lld %lld %lld\n", st.status, (long long)st.n_fwd, (long long)st.n_rev,
         (long long)st.n_fwd_kept, (long long)st.n_rev_kept, (long long)st.n_pairs);
  return 0;
}

static int writecalls_mode(char** argv) {
  const long long n = atoll(argv[2]);
  unsigned long long x = (unsigned long long)atoll(argv[3]) * 2654435761ull + 1;
  uint32_t* calls = (uint32_t*)malloc(sizeof(uint32_t) * 4 * (size_t)(n > 0 ? n : 1));
  const char b[6] = {'A', 'C', 'G', 'T', 'N', 'X'};
  for (long long k = 0; k < n; ++k) {
    x ^= x << 13; x ^= x >> 7; x ^= x << 17;
    const uint32_t tot = 1 + (uint32_t)(x % 2000000000ull);
    calls[4 * k] = (uint32_t)b[x % 5] | ((uint32_t)b[(x >> 8) % 5] << 8) | ((uint32_t)b[(x >> 16) % 6] << 16);
    calls[4 * k + 1] = 1 + (uint32_t)((x >> 20) % tot);
    calls[4 * k + 2] = (uint32_t)((x >> 30) % 1000);
    calls[4 * k + 3] = tot;
  }
  char msg[256];
  const int rc = mpc_write_calls(calls, n, argv[4], argv[5], argv[6], 4, msg, 256);
  free(calls);
  printf("%d\n", rc);
  return 0;
}

int main(int argc, char** argv) {
  if (argc == 5 && !strcmp(argv[1], "pseudopair")) return pseudopair_mode(argv);
  if (argc == 7 && !strcmp(argv[1], "writecalls")) return writecalls_mode(argv);
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
