// RTen's thread-pool size, restated for the places where it changes numerics
// (the gemv column blocks, src/gemm.rs:676).
//
// src/threading.rs:41-62 sizes the rayon pool to num_cpus::get_physical(),
// or to RTEN_NUM_THREADS parsed as usize and clamped to [1, num_cpus::get()]
// (a value that does not parse falls back to the physical count).  num_cpus
// 1.16 (Cargo.lock:268-269) on Linux:
//  - get():          CPUs in the sched affinity mask, capped by a cgroup CPU
//                    quota ceil(quota / period) when one is set;
//  - get_physical(): the sum of "cpu cores" over the distinct "physical id"s
//                    of /proc/cpuinfo, or get() when that finds nothing.
#pragma once

#include <sched.h>
#include <unistd.h>

#include <cerrno>
#include <climits>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <string>

namespace rtenhip {

inline int cgroup_cpu_quota() {
  // cgroup v2 "cpu.max" ("max 100000" = no quota), then v1 cfs quota / period.
  std::ifstream f2("/sys/fs/cgroup/cpu.max");
  std::string q, p;
  if (f2 >> q >> p) {
    if (q == "max") return 0;
    const double qv = atof(q.c_str()), pv = atof(p.c_str());
    return qv > 0 && pv > 0 ? (int)std::ceil(qv / pv) : 0;
  }
  std::ifstream fq("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), fp("/sys/fs/cgroup/cpu/cpu.cfs_period_us");
  long long qv = -1, pv = 0;
  if (fq >> qv && fp >> pv && qv > 0 && pv > 0) return (int)((qv + pv - 1) / pv);
  return 0;
}

// num_cpus::get()
inline int logical_cpus() {
  int n = 0;
  cpu_set_t set;
  CPU_ZERO(&set);
  if (sched_getaffinity(0, sizeof(set), &set) == 0) {
    n = CPU_COUNT(&set);
  } else {
    long c = sysconf(_SC_NPROCESSORS_ONLN);
    n = c < 1 ? 1 : (int)c;
  }
  const int quota = cgroup_cpu_quota();
  if (quota > 0 && quota < n) n = quota;
  return n < 1 ? 1 : n;
}

// num_cpus::get_physical()
inline int physical_cpus() {
  std::ifstream f("/proc/cpuinfo");
  std::map<unsigned, int> cores_of;  // physical id -> "cpu cores"
  unsigned physid = 0;
  int cores = 0, changes = 0;
  std::string line;
  while (std::getline(f, line)) {
    const size_t colon = line.find(':');
    if (colon == std::string::npos) continue;
    std::string key = line.substr(0, colon), val = line.substr(colon + 1);
    auto trim = [](std::string& s) {
      const size_t a = s.find_first_not_of(" \t"), b = s.find_last_not_of(" \t");
      s = a == std::string::npos ? "" : s.substr(a, b - a + 1);
    };
    trim(key);
    trim(val);
    char* end = nullptr;
    if (key == "physical id") {
      physid = (unsigned)strtoul(val.c_str(), &end, 10);
      if (val.empty() || *end) break;
      changes++;
    } else if (key == "cpu cores") {
      cores = (int)strtol(val.c_str(), &end, 10);
      if (val.empty() || *end) break;
      changes++;
    }
    if (changes == 2) {
      cores_of[physid] = cores;
      changes = 0;
    }
  }
  int total = 0;
  for (auto& kv : cores_of) total += kv.second;
  return total > 0 ? total : logical_cpus();
}

// rten::threading::thread_pool() size.
inline int rten_num_threads() {
  const char* s = getenv("RTEN_NUM_THREADS");
  if (s) {
    // Rust usize::from_str: decimal digits only (an optional leading '+'),
    // no whitespace, no sign '-'; overflow is an error.
    const char* p = s[0] == '+' ? s + 1 : s;
    bool ok = *p != 0;
    unsigned long long v = 0;
    for (const char* c = p; ok && *c; c++) {
      if (*c < '0' || *c > '9') ok = false;
      else if (v > (ULLONG_MAX - 9) / 10) ok = false;
      else v = v * 10 + (unsigned)(*c - '0');
    }
    if (ok) {
      const int lg = logical_cpus();
      return v < 1 ? 1 : v > (unsigned long long)lg ? lg : (int)v;
    }
  }
  return physical_cpus();
}

}  // namespace rtenhip
