// host_threads.h -- default worker-thread count of the host-side libraries.
#pragma once
#include <sched.h>

#include <cstdlib>
#include <thread>

namespace mpc_host {
// OMP_NUM_THREADS when set (the GPU pool sets it to the job's CPU share), else
// the CPUs this process may run on.  Not hardware_concurrency() alone: that
// counts the whole machine, and a shared box gives a job a fraction of it.
inline int host_threads() {
  if (const char* e = getenv("OMP_NUM_THREADS")) {
    const int v = atoi(e);
    if (v > 0) return v;
  }
  cpu_set_t cs;
  if (sched_getaffinity(0, sizeof(cs), &cs) == 0 && CPU_COUNT(&cs) > 0) return CPU_COUNT(&cs);
  const unsigned hw = std::thread::hardware_concurrency();
  return hw ? (int)hw : 4;
}
}  // namespace mpc_host
