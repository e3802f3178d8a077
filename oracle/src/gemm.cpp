// CPU restatement of RTen's GEMM engine (test infrastructure; see rten_oracle.h).
//
// Follows src/gemm.rs:546-1050 (block sizes, gemm_impl, gemm_block, gemv),
// src/gemm/packing.rs:20-186 (panel packing) and src/gemm/kernels.rs:26-316 +
// src/gemm/kernels/x86_64.rs:19-130 (FmaKernel, MR=6 NR=16, simd_gemv*).
#include <immintrin.h>
#include <omp.h>

#include <algorithm>
#include <cstdlib>
#include <mutex>
#include <map>
#include <string>
#include <cctype>
#include <cstdio>
#include <cstring>
#include <sched.h>
#include <unistd.h>

#include "common.h"

namespace orc {

static thread_local std::string g_err;
static thread_local int g_err_code = 0;

void set_error(int code, const std::string& msg) {
  g_err_code = code;
  g_err = msg;
}
int fail(int code, const char* msg) {
  set_error(code, msg);
  return code;
}

static int g_threads = 0;
static std::once_flag g_threads_once;

// num_cpus 1.16 (Cargo.lock:268-269) on Linux.  get(): CPUs in the affinity
// mask, capped by a cgroup CPU quota ceil(quota / period).
static int logical_cpus() {
  cpu_set_t set;
  CPU_ZERO(&set);
  int n = sched_getaffinity(0, sizeof(set), &set) == 0 ? CPU_COUNT(&set)
                                                       : (int)std::max(1L, sysconf(_SC_NPROCESSORS_ONLN));
  long long q = -1, p = 0;
  char mx[32] = {0};
  if (FILE* f = fopen("/sys/fs/cgroup/cpu.max", "r")) {
    if (fscanf(f, "%31s %lld", mx, &p) == 2 && strcmp(mx, "max") != 0) q = atoll(mx);
    fclose(f);
  } else if (FILE* fq = fopen("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", "r")) {
    if (fscanf(fq, "%lld", &q) != 1) q = -1;
    fclose(fq);
    if (FILE* fp = fopen("/sys/fs/cgroup/cpu/cpu.cfs_period_us", "r")) {
      if (fscanf(fp, "%lld", &p) != 1) p = 0;
      fclose(fp);
    }
  }
  if (q > 0 && p > 0) n = std::min<long long>(n, (q + p - 1) / p);
  return std::max(1, n);
}

// get_physical(): sum of "cpu cores" per distinct "physical id" in
// /proc/cpuinfo (pairs taken as they complete), else get().
static int physical_cpus() {
  std::map<unsigned, int> per_socket;
  FILE* f = fopen("/proc/cpuinfo", "r");
  if (f) {
    char line[512];
    unsigned pid = 0;
    int cores = 0, seen = 0;
    while (fgets(line, sizeof line, f)) {
      char* colon = strchr(line, ':');
      if (!colon) continue;
      *colon = 0;
      std::string key(line), val(colon + 1);
      while (!key.empty() && isspace((unsigned char)key.back())) key.pop_back();
      while (!val.empty() && isspace((unsigned char)val.back())) val.pop_back();
      while (!val.empty() && isspace((unsigned char)val.front())) val.erase(0, 1);
      char* end = nullptr;
      if (key == "physical id") {
        pid = (unsigned)strtoul(val.c_str(), &end, 10);
        if (val.empty() || *end) break;
        seen++;
      } else if (key == "cpu cores") {
        cores = (int)strtol(val.c_str(), &end, 10);
        if (val.empty() || *end) break;
        seen++;
      }
      if (seen == 2) {
        per_socket[pid] = cores;
        seen = 0;
      }
    }
    fclose(f);
  }
  int total = 0;
  for (auto& kv : per_socket) total += kv.second;
  return total > 0 ? total : logical_cpus();
}

// src/threading.rs:41-62: physical cores, or RTEN_NUM_THREADS (a usize)
// clamped to [1, logical]; an unparsable value means physical.
static int resolve_threads() {
  const char* s = getenv("RTEN_NUM_THREADS");
  if (s) {
    const char* d = *s == '+' ? s + 1 : s;
    bool ok = *d != 0 && strlen(d) < 19;
    for (const char* c = d; ok && *c; c++) ok = *c >= '0' && *c <= '9';
    if (ok) return (int)std::max(1LL, std::min<long long>(atoll(d), logical_cpus()));
  }
  return physical_cpus();
}

int threads() {
  std::call_once(g_threads_once, [] {
    if (g_threads == 0) g_threads = resolve_threads();
    omp_set_num_threads(g_threads);
  });
  return g_threads;
}

int64_t numel(const int64_t* shape, int ndim) {
  int64_t n = 1;
  for (int i = 0; i < ndim; i++) n *= shape[i];
  return n;
}

static constexpr int MR = 6;   // FmaKernel::MR (x86_64.rs:27)
static constexpr int NR = 16;  // FmaKernel::NR (x86_64.rs:31)

static inline int64_t next_mult(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// src/gemm.rs:546-571
static int64_t depth_block_size(int64_t a_cols) { return std::min<int64_t>(256, a_cols); }
static int64_t col_block_size(int64_t b_cols, int64_t nr, int par) {
  int64_t lower = std::min<int64_t>(128, b_cols);
  int64_t unrounded = std::min<int64_t>(std::max<int64_t>(b_cols / par, lower), 1024);
  return next_mult(unrounded, nr);
}
static int64_t row_block_size(int64_t a_rows, int64_t mr) {
  return next_mult(std::min<int64_t>(64, a_rows), mr);
}

// pack_a_block (packing.rs:20-90): MR-row panels, column-major, zero padded.
static void pack_a_block(float* out, const Mat& a, int64_t r0, int64_t r1, int64_t c0,
                         int64_t c1) {
  int64_t rows = r1 - r0, cols = c1 - c0;
  int64_t n_panels = next_mult(rows, MR) / MR;
  for (int64_t p = 0; p < n_panels; p++) {
    float* po = out + p * cols * MR;
    for (int64_t c = 0; c < cols; c++)
      for (int r = 0; r < MR; r++) {
        int64_t ar = r0 + p * MR + r;
        po[c * MR + r] = ar < r1 ? a.at(ar, c0 + c) : 0.f;
      }
  }
}

// pack_b_block (packing.rs:106-186): NR-col panels, row-major, zero padded.
static void pack_b_block(float* out, const Mat& b, int64_t r0, int64_t r1, int64_t c0,
                         int64_t c1) {
  int64_t rows = r1 - r0, cols = c1 - c0;
  int64_t n_panels = next_mult(cols, NR) / NR;
  for (int64_t p = 0; p < n_panels; p++) {
    float* po = out + p * rows * NR;
    int64_t pc = c0 + p * NR;
    bool full = c1 - pc >= NR;
    for (int64_t r = 0; r < rows; r++) {
      const float* src = b.data + (r0 + r) * b.rs + pc * b.cs;
      if (full && b.cs == 1) {
        memcpy(po + r * NR, src, NR * sizeof(float));
      } else {
        for (int c = 0; c < NR; c++) po[r * NR + c] = (pc + c < c1) ? src[c * b.cs] : 0.f;
      }
    }
  }
}

// simd_gemm::<__m256, 6, 2> (kernels.rs:206-316): one fma chain per output
// element from +0 over `depth`, then the alpha/beta store variants.  The
// first depth - 1 steps run unrolled x4 with a prefetch of the next step's B
// row (kernels.rs:226-245, unroll_loop! + S::prefetch); the last step follows
// a write prefetch of the tile (kernels.rs:247-268).  The fma order per
// element is the same k-ordered chain either way.
__attribute__((target("avx2,fma"), always_inline)) static inline void k6x16_step(__m256 (&acc)[MR][2], const float* a,
                                                                                  const float* b, int64_t k) {
  const __m256 b0 = _mm256_loadu_ps(b + k * NR);
  const __m256 b1 = _mm256_loadu_ps(b + k * NR + 8);
  const float* ak = a + k * MR;
  for (int i = 0; i < MR; i++) {
    const __m256 av = _mm256_set1_ps(ak[i]);
    acc[i][0] = _mm256_fmadd_ps(av, b0, acc[i][0]);
    acc[i][1] = _mm256_fmadd_ps(av, b1, acc[i][1]);
  }
}

__attribute__((target("avx2,fma"))) static void kernel_6x16(float* tile, int64_t tile_rs,
                                                            const float* a, const float* b,
                                                            int64_t depth, float alpha,
                                                            float beta) {
  __m256 acc[MR][2];
  for (int i = 0; i < MR; i++) acc[i][0] = acc[i][1] = _mm256_setzero_ps();
  const int64_t body = depth - 1;
  int64_t k = 0;
  for (; k + 4 <= body; k += 4) {
    _mm_prefetch((const char*)(b + (k + 1) * NR), _MM_HINT_T0);
    k6x16_step(acc, a, b, k);
    _mm_prefetch((const char*)(b + (k + 2) * NR), _MM_HINT_T0);
    k6x16_step(acc, a, b, k + 1);
    _mm_prefetch((const char*)(b + (k + 3) * NR), _MM_HINT_T0);
    k6x16_step(acc, a, b, k + 2);
    _mm_prefetch((const char*)(b + (k + 4) * NR), _MM_HINT_T0);
    k6x16_step(acc, a, b, k + 3);
  }
  for (; k < body; k++) {
    _mm_prefetch((const char*)(b + (k + 1) * NR), _MM_HINT_T0);
    k6x16_step(acc, a, b, k);
  }
  for (int i = 0; i < MR; i++) _mm_prefetch((const char*)(tile + i * tile_rs), _MM_HINT_T0);
  if (depth > 0) k6x16_step(acc, a, b, depth - 1);
  if (beta == 0.f && alpha == 1.f) {
    for (int i = 0; i < MR; i++) {
      _mm256_storeu_ps(tile + i * tile_rs, acc[i][0]);
      _mm256_storeu_ps(tile + i * tile_rs + 8, acc[i][1]);
    }
  } else if (beta == 1.f && alpha == 1.f) {
    for (int i = 0; i < MR; i++)
      for (int j = 0; j < 2; j++) {
        float* p = tile + i * tile_rs + j * 8;
        _mm256_storeu_ps(p, _mm256_add_ps(_mm256_loadu_ps(p), acc[i][j]));
      }
  } else if (beta == 0.f) {
    __m256 al = _mm256_set1_ps(alpha);
    for (int i = 0; i < MR; i++)
      for (int j = 0; j < 2; j++)
        _mm256_storeu_ps(tile + i * tile_rs + j * 8, _mm256_mul_ps(acc[i][j], al));
  } else {
    __m256 al = _mm256_set1_ps(alpha), be = _mm256_set1_ps(beta);
    for (int i = 0; i < MR; i++)
      for (int j = 0; j < 2; j++) {
        float* p = tile + i * tile_rs + j * 8;
        __m256 o = _mm256_mul_ps(_mm256_loadu_ps(p), be);
        _mm256_storeu_ps(p, _mm256_fmadd_ps(acc[i][j], al, o));
      }
  }
}

// gemm_block (src/gemm.rs:941-1050).
static void gemm_block(float* out, int64_t out_rs, int64_t out_rows, int64_t out_cols,
                       int64_t col_tile0, int64_t col_tile1, int64_t row_tile0, int64_t row_tile1,
                       bool first_update, const float* packed_a, const float* packed_b,
                       int64_t panel_len, float alpha, float beta, const float* bias) {
  int64_t b_panel = panel_len * NR, a_panel = MR * panel_len;
  for (int64_t ct = col_tile0; ct < col_tile1; ct++) {
    const float* bp = packed_b + (ct - col_tile0) * b_panel;
    for (int64_t rt = row_tile0; rt < row_tile1; rt++) {
      const float* ap = packed_a + (rt - row_tile0) * a_panel;
      int64_t r0 = rt * MR, c0 = ct * NR;
      int64_t used_rows = std::min<int64_t>(out_rows - r0, MR);
      int64_t used_cols = std::min<int64_t>(out_cols - c0, NR);
      float* tp = out + r0 * out_rs + c0;
      if (used_rows == MR && used_cols == NR) {
        kernel_6x16(tp, out_rs, ap, bp, panel_len, alpha, beta);
      } else {
        float tmp[MR * NR];
        kernel_6x16(tmp, NR, ap, bp, panel_len, alpha, 0.f);
        for (int64_t i = 0; i < used_rows; i++)
          for (int64_t j = 0; j < used_cols; j++) {
            float* o = tp + i * out_rs + j;
            float t = beta == 0.f ? 0.f : *o;
            *o = beta * t + tmp[i * NR + j];
          }
      }
      if (bias && first_update) {
        for (int64_t i = 0; i < used_rows; i++)
          for (int64_t j = 0; j < used_cols; j++) tp[i * out_rs + j] += bias[r0 + i];
      }
    }
  }
}

// __m256::sum (rten-simd/src/arch/x86_64.rs:236-248).
static inline float hsum8(const float v[8]) {
  float s4[4], s2[2];
  for (int i = 0; i < 4; i++) s4[i] = v[i] + v[i + 4];
  for (int i = 0; i < 2; i++) s2[i] = s4[i] + s4[i + 2];
  return s2[0] + s2[1];
}

// simd_gemv_fallback (kernels.rs:174-194).
static void gemv_fallback(float* out, const float* a, const Mat& b, float alpha, float beta) {
  for (int64_t c = 0; c < b.cols; c++) {
    float acc = 0.f;
    for (int64_t k = 0; k < b.rows; k++) acc = fmaf(a[k], b.at(k, c), acc);
    acc *= alpha;
    if (beta == 0.f)
      out[c] = acc;
    else
      out[c] = acc + beta * out[c];
  }
}

// simd_gemv_transposed (kernels.rs:109-167), S::LEN = 8, COL_TILE = 8.
static void gemv_transposed(float* out, const float* a, const Mat& b, float alpha, float beta) {
  const int64_t L = 8, CT = 8;
  int64_t depth = b.rows;
  int64_t n_full_cols = b.cols / CT * CT, n_full_depth = depth / L * L;
  for (int64_t c0 = 0; c0 < n_full_cols; c0 += CT) {
    float accv[CT][8];
    for (int i = 0; i < CT; i++)
      for (int j = 0; j < 8; j++) accv[i][j] = 0.f;
    for (int64_t d0 = 0; d0 < n_full_depth; d0 += L)
      for (int i = 0; i < CT; i++) {
        const float* col = b.data + (c0 + i) * b.cs;
        for (int j = 0; j < 8; j++) accv[i][j] = fmaf(a[d0 + j], col[d0 + j], accv[i][j]);
      }
    float acc[CT];
    for (int i = 0; i < CT; i++) acc[i] = hsum8(accv[i]);
    for (int64_t k = n_full_depth; k < depth; k++)
      for (int i = 0; i < CT; i++) acc[i] = fmaf(a[k], b.data[(c0 + i) * b.cs + k], acc[i]);
    for (int i = 0; i < CT; i++) {
      if (beta == 0.f)
        out[c0 + i] = alpha * acc[i];
      else
        out[c0 + i] = alpha * acc[i] + beta * out[c0 + i];
    }
  }
  if (n_full_cols < b.cols) {
    Mat rem{b.data + n_full_cols * b.cs, b.rows, b.cols - n_full_cols, b.rs, b.cs};
    gemv_fallback(out + n_full_cols, a, rem, alpha, beta);
  }
}

// simd_gemv::<__m256, 4> (kernels.rs:26-103).
static void gemv_kernel(float* out, const float* a, const Mat& b, float alpha, float beta) {
  if (b.rs == 1) return gemv_transposed(out, a, b, alpha, beta);
  if (b.cs != 1) return gemv_fallback(out, a, b, alpha, beta);
  const int64_t T = 32;
  int64_t n_full = b.cols / T * T;
  for (int64_t c0 = 0; c0 < n_full; c0 += T) {
    float acc[T];
    for (int j = 0; j < T; j++) acc[j] = 0.f;
    for (int64_t k = 0; k < b.rows; k++) {
      const float* row = b.data + k * b.rs + c0;
      for (int j = 0; j < T; j++) acc[j] = fmaf(a[k], row[j], acc[j]);
    }
    if (alpha != 1.f)
      for (int j = 0; j < T; j++) acc[j] = acc[j] * alpha;
    for (int j = 0; j < T; j++) {
      if (beta == 0.f)
        out[c0 + j] = acc[j];
      else if (beta == 1.f)
        out[c0 + j] = out[c0 + j] + acc[j];
      else
        out[c0 + j] = fmaf(out[c0 + j], beta, acc[j]);
    }
  }
  for (int64_t c = n_full; c < b.cols; c++) {
    float acc = 0.f;
    for (int64_t k = 0; k < b.rows; k++) acc += a[k] * b.data[k * b.rs + c];
    float t = beta == 0.f ? 0.f : out[c];
    out[c] = beta * t + acc * alpha;
  }
}

// gemv (src/gemm.rs:651-704).
static void gemv(float* out, const Mat& a, const Mat& b, float alpha, float beta,
                 const float* bias, bool serial) {
  int64_t K = a.cols, N = b.cols;
  std::vector<float> av(K);
  for (int64_t k = 0; k < K; k++) av[k] = a.at(0, k);
  int par = threads();
  int64_t bbs = std::max<int64_t>((N + par - 1) / par, 128);
  int64_t kbs = b.rs == 1 ? 512 : 8;
  int64_t n_blocks = (N + bbs - 1) / bbs;
#pragma omp parallel for schedule(dynamic, 1) if (!serial && n_blocks > 1)
  for (int64_t cb = 0; cb < n_blocks; cb++) {
    int64_t c0 = cb * bbs, c1 = std::min(N, c0 + bbs);
    float eb = beta;
    for (int64_t k0 = 0; k0 < K; k0 += kbs) {
      int64_t k1 = std::min(K, k0 + kbs);
      Mat bb{b.data + k0 * b.rs + c0 * b.cs, k1 - k0, c1 - c0, b.rs, b.cs};
      gemv_kernel(out + c0, av.data() + k0, bb, alpha, eb);
      eb = 1.f;
    }
    if (bias)
      for (int64_t c = c0; c < c1; c++) out[c] += bias[0];
  }
}

void gemm_impl(float* out, int64_t out_rs, const Mat& a, const Mat* b, const VirtualB* vb,
               float alpha, float beta, const float* bias, bool serial) {
  int64_t M = a.rows, K = a.cols, N = b ? b->cols : vb->cols();
  if (M == 0 || N == 0) return;
  if (K == 0) {
    for (int64_t r = 0; r < M; r++)
      for (int64_t c = 0; c < N; c++) {
        float& x = out[r * out_rs + c];
        float t = beta == 0.f ? 0.f : x;
        x = beta * t;
      }
    return;
  }
  if (M == 1 && b) return gemv(out, a, *b, alpha, beta, bias, serial);

  int par = threads();
  int64_t nc = col_block_size(N, NR, par);
  int64_t mc = row_block_size(M, MR);
  int64_t kc = depth_block_size(K);
  int64_t n_col_blocks = (N + nc - 1) / nc, n_row_blocks = (M + mc - 1) / mc;
  int64_t b_panel_cap = next_mult(nc, NR) * kc;
  std::vector<float> packed_b(n_col_blocks * b_panel_cap);
  bool parallel = !serial && par > 1;

  for (int64_t d0 = 0; d0 < K; d0 += kc) {
    int64_t d1 = std::min(K, d0 + kc), plen = d1 - d0;
    float eff_beta = d0 == 0 ? beta : 1.f;
#pragma omp parallel for schedule(dynamic, 1) if (parallel && n_col_blocks > 1)
    for (int64_t cb = 0; cb < n_col_blocks; cb++) {
      int64_t c0 = cb * nc, c1 = std::min(N, c0 + nc);
      float* pb = packed_b.data() + cb * b_panel_cap;
      if (b)
        pack_b_block(pb, *b, d0, d1, c0, c1);
      else
        vb->pack_b(pb, NR, d0, d1, c0, c1);
    }
    int64_t n_work = n_col_blocks * n_row_blocks;
#pragma omp parallel if (parallel && n_work > 1)
    {
      std::vector<float> packed_a(next_mult(mc, MR) * kc);
#pragma omp for schedule(dynamic, 1)
      for (int64_t w = 0; w < n_work; w++) {
        int64_t cb = w / n_row_blocks, rb = w % n_row_blocks;
        int64_t c0 = cb * nc, c1 = std::min(N, c0 + nc);
        int64_t r0 = rb * mc, r1 = std::min(M, r0 + mc);
        pack_a_block(packed_a.data(), a, r0, r1, d0, d1);
        gemm_block(out, out_rs, M, N, c0 / NR, (c1 + NR - 1) / NR, r0 / MR, (r1 + MR - 1) / MR,
                   d0 == 0, packed_a.data(), packed_b.data() + cb * b_panel_cap, plen, alpha,
                   eff_beta, bias);
      }
    }
  }
}

}  // namespace orc

using namespace orc;

extern "C" {

const char* orc_last_error(void) { return g_err.c_str(); }

int orc_num_threads(void) { return threads(); }
void orc_set_num_threads(int n) {
  threads();
  g_threads = std::max(1, n);
  omp_set_num_threads(g_threads);
}
int orc_reset_threads(void) {
  threads();
  g_threads = resolve_threads();
  omp_set_num_threads(g_threads);
  return g_threads;
}
void orc_cpu_counts(int* logical, int* physical) {
  if (logical) *logical = logical_cpus();
  if (physical) *physical = physical_cpus();
}

void orc_xorshift_fill(uint64_t* state, float* out, int64_t n) {
  // rten-tensor/src/rng.rs:17-35
  const float scale = 1.0f / (float)(1ull << 40);
  uint64_t s = *state;
  for (int64_t i = 0; i < n; i++) {
    s ^= s << 13;
    s ^= s >> 7;
    s ^= s << 17;
    uint64_t v = s >> (64 - 40);
    out[i] = (float)v * scale;
  }
  *state = s;
}

int orc_gemm(float* out, int64_t out_rs, const float* a, int64_t a_rs, int64_t a_cs,
             const float* b, int64_t b_rs, int64_t b_cs, int64_t m, int64_t n, int64_t k,
             float alpha, float beta, const float* bias) {
  Mat A{a, m, k, a_rs, a_cs}, B{b, k, n, b_rs, b_cs};
  gemm_impl(out, out_rs, A, &B, nullptr, alpha, beta, bias, false);
  return ORC_OK;
}

// Test helper: reference_gemm (src/gemm.rs:1126-1147), f32 accumulation.
void orc_reference_gemm(float* out, const float* a, const float* b, int64_t m, int64_t n,
                        int64_t k, float alpha, float beta, const float* bias) {
  for (int64_t r = 0; r < m; r++)
    for (int64_t c = 0; c < n; c++) {
      float acc = 0.f;
      for (int64_t i = 0; i < k; i++) acc += a[r * k + i] * b[i * n + c];
      out[r * n + c] = alpha * acc + beta * out[r * n + c] + (bias ? bias[r] : 0.f);
    }
}

}  // extern "C"
