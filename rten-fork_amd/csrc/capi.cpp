// C ABI entry points (include/rten_hip.h): host-side validation and dispatch
// for each operator, mirroring the reference's Operator::run bodies
// (shape checks, error kinds and messages) and launching the HIP kernels.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>
#include <vector>

#include "common.h"
#include "ctx.h"
#include "gemm_dma.h"
#include "threads.h"

namespace rtenhip {

static thread_local std::string g_err;
static thread_local int g_err_code = 0;

void set_error(int code, const std::string& msg) {
  g_err_code = code;
  g_err = msg;
}
rtenhip_status fail(rtenhip_status code, const char* msg) {
  set_error(code, msg);
  return code;
}
rtenhip_status hip_fail(hipError_t e, const char* where) {
  set_error(RTENHIP_HIP_ERROR, std::string("HIP error ") + hipGetErrorString(e) + " at " + where);
  return RTENHIP_HIP_ERROR;
}

hipStream_t stream_of(rtenhip_ctx* ctx) { return reinterpret_cast<Ctx*>(ctx)->stream; }

Ctx::Ctx(int dev) : device(dev), ref_threads(rten_num_threads()) {}

Ctx::~Ctx() {
  if (exec_stream) {
    (void)hipStreamSynchronize(exec_stream);
    if (owns_exec) (void)hipStreamDestroy(exec_stream);
  }
  for (auto& kv : ktabs) (void)hipFree(kv.second);
  for (auto& kv : dtabs) (void)hipFree(kv.second);
  for (auto& kv : packed_cache) (void)hipFree(kv.second);
  if (counters) (void)hipFree(counters);
  for (int i = 0; i < NSLOTS; i++)
    if (slots[i]) (void)hipFree(slots[i]);
}

float* Ctx::scratch_floats(size_t n, size_t slot) {
  size_t need = n * sizeof(float);
  if (slot >= (size_t)NSLOTS) return nullptr;
  if (scratch_log) {
    size_t& m = (*scratch_log)[slot];
    m = std::max(m, n);
  }
  if (need > slot_cap[slot] || !slots[slot]) {
    void* p = nullptr;
    size_t cap = need + (need >> 2) + 256;
    if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
    if (hipMalloc(&p, cap) != hipSuccess) return nullptr;
    if (slots[slot]) (void)hipFree(slots[slot]);
    slots[slot] = p;
    slot_cap[slot] = cap;
    scratch_gen++;
  }
  return static_cast<float*>(slots[slot]);
}

int* Ctx::split_counters(size_t n) {
  if (scratch_log) {
    size_t& m = (*scratch_log)[NSLOTS];
    m = std::max(m, n);
  }
  if (n > counters_cap || !counters) {
    if (hipStreamSynchronize(stream) != hipSuccess) return nullptr;
    if (counters) (void)hipFree(counters);
    counters = nullptr;
    size_t cap = n + 64;
    if (hipMalloc(&counters, cap * sizeof(int)) != hipSuccess) return nullptr;
    // Ordered on the stream the split kernels run on: a plain hipMemset is not
    // ordered with a non-blocking stream.
    if (hipMemsetAsync(counters, 0, cap * sizeof(int), stream) != hipSuccess) return nullptr;
    counters_cap = cap;
    scratch_gen++;
  }
  return counters;
}

bool Ctx::reserve_scratch(const std::map<size_t, size_t>& need) {
  for (auto& kv : need) {
    if (kv.first == (size_t)NSLOTS) {
      if (!split_counters(kv.second)) return false;
    } else if (!scratch_floats(kv.second, kv.first)) {
      return false;
    }
  }
  return true;
}

const int* Ctx::dtab(int C, int H, int W, int kh, int kw, int dh, int dw) {
  auto key = std::make_tuple(C, H, W, kh, kw, dh, dw);
  std::lock_guard<std::mutex> g(mu);
  auto it = dtabs.find(key);
  if (it != dtabs.end()) return it->second;
  // Byte offsets, padded with out-of-range entries to a whole number of the
  // largest K tile so the kernel never bounds-checks k.
  const size_t K = (size_t)C * kh * kw;
  std::vector<int> tab((K + DMA_KTAB_PAD - 1) / DMA_KTAB_PAD * DMA_KTAB_PAD, (int)DMA_OOB);
  size_t r = 0;
  for (int c = 0; c < C; c++)
    for (int ky = 0; ky < kh; ky++)
      for (int kx = 0; kx < kw; kx++) tab[r++] = (c * H * W + ky * dh * W + kx * dw) * 4;
  int* d = nullptr;
  if (hipMalloc(&d, tab.size() * sizeof(int)) != hipSuccess) return nullptr;
  if (hipMemcpy(d, tab.data(), tab.size() * sizeof(int), hipMemcpyHostToDevice) != hipSuccess)
    return nullptr;
  dtabs[key] = d;
  return d;
}

bool conv_dma_eligible(int64_t N, int64_t C, int64_t Hp, int64_t Wp, int64_t O, int64_t groups,
                       int64_t K) {
  // 32-bit buffer offsets: the whole (padded) input must stay below 2 GiB.
  const int64_t x_elems = N * C * Hp * Wp;
  return x_elems < (int64_t(1) << 29) && K >= 1 && O / groups >= 1;
}

// DmaDesc of group g of a conv (everything but the split / persistence
// fields).  lat: the latency GEMM's addressing (lat-packed A, and for 1x1
// kernels koff(k) = k * Hp * Wp without a table).
static void fill_conv_desc(const ConvDmaArgs& a, int64_t g, bool lat, const DmaTile& tile, const int* tab,
                           DmaDesc& d) {
  const int64_t opg = a.O / a.groups, ipg = a.C / a.groups;
  const int64_t K = ipg * a.kh * a.kw, P = a.oh * a.ow;
  const int64_t per_group = lat ? lat_packed_floats((int)opg, (int)K) : packed_a_floats((int)opg, (int)K, tile);
  const int64_t x_total = a.N * a.C * a.Hp * a.Wp;
  d = DmaDesc{};
  d.M = (int)opg;
  d.N = (int)(a.N * P);
  d.K = (int)K;
  d.tile = tile;
  d.apk = a.packed_w + g * per_group;
  d.x = a.xin + g * ipg * a.Hp * a.Wp;
  d.x_bytes = (uint32_t)((x_total - g * ipg * a.Hp * a.Wp) * 4);
  d.x_img = a.C * a.Hp * a.Wp;
  d.ystride = a.sh * a.Wp;
  d.xstride = a.sw;
  d.OW = (int)a.ow;
  d.P = (int)P;
  d.fdOW = make_fastdiv((uint32_t)a.ow);
  d.fdP = make_fastdiv((uint32_t)P);
  d.ktab4 = tab;
  d.out_img = a.y_img;
  d.out_c = P;  // channel stride of an unpadded output plane
  d.out_row = a.ow;
  d.out_off = 0;
  if (a.y_row) {
    // padded output planes: (oh + 2*pad) x y_row, interior at y_off
    d.out_c = a.y_img / a.O;
    d.out_row = a.y_row;
    d.out_off = a.y_off;
  }
  d.out = a.y + g * opg * d.out_c;
  d.residual = a.residual ? a.residual + g * opg * P : nullptr;
  d.res_img = a.O * P;
  d.res_c = P;
  d.bias = a.bias ? a.bias + g * opg : nullptr;
  d.bn = a.bn ? a.bn + g * opg : nullptr;
  d.bn_c = (int)a.bn_c;
  d.alpha = 1.f;
  d.beta = 0.f;
  d.vec4 = (P % 4 == 0 && d.out_c == P && d.out_row == a.ow && d.out_off == 0 && d.out_img % 4 == 0 &&
            d.res_img % 4 == 0 && g * opg * P % 4 == 0 && ((uintptr_t)a.y % 16) == 0 &&
            (!a.residual || ((uintptr_t)a.residual % 16) == 0))
               ? 1
               : 0;
  d.act = a.act;
  d.act_lo = a.lo;
  d.act_hi = a.hi;
  if (lat && a.kh == 1 && a.kw == 1) d.kstride = (int)(a.Hp * a.Wp);
  static const bool lat_ktab = getenv("RTENHIP_LAT_KTAB") != nullptr;  // A/B experiments: table offsets
  static const int lat_dbg = getenv("RTENHIP_LAT_DBG") ? atoi(getenv("RTENHIP_LAT_DBG")) : 0;
  if (lat) d.dbg = lat_dbg;
  if (lat && a.kh == 3 && a.kw == 3 && !lat_ktab) {
    // Same offsets as the table (Ctx::dtab), formed in the kernel.
    d.k3x3 = 1;
    d.kt_plane = (int)(a.Hp * a.Wp);
    d.kt_row = (int)(a.dh * a.Wp);
    d.kt_col = (int)a.dw;
  }
}

// 16-byte B copies: pointwise stride-1 convs (B[k][n] = x[img][k][p],
// linear in k) whose 4-pixel groups stay inside one image.
static void set_conv_bvec(const ConvDmaArgs& a, int cfg, const DmaTile& tile, DmaDesc& d) {
  const int64_t P = a.oh * a.ow;
  const bool pointwise = a.kh == 1 && a.kw == 1 && a.sh == 1 && a.sw == 1 && a.Hp == a.oh && a.Wp == a.ow;
  if (pointwise && dma_cfg_bvec(cfg) && P % 4 == 0 && d.K % tile.bk == 0 && (a.C * a.Hp * a.Wp) % 4 == 0 &&
      ((uintptr_t)d.x % 16) == 0) {
    d.bvec = 1;
    d.kstride = (int)(a.Hp * a.Wp);
  }
}

// The latency GEMM's K-block workspace and 16-byte B copies for variant v
// (gemm_lat2 / gemm_lat3, variants 7x / 8x: pointwise stride-1 convs whose
// 4-column groups stay inside one image).
static rtenhip_status lat_conv_split_bvec(const ConvDmaArgs& a, int v, DmaDesc& d) {
  const DmaSplit sp = lat_split_plan(d.M, d.N, d.K, v);
  if (sp.split_tiles > 0) {
    if (!a.split || !a.ws || !a.counters || sp.ws_floats > a.ws_cap || sp.counters > a.cnt_cap)
      return fail(RTENHIP_INVALID_VALUE, "latency conv: K-block workspace missing or too small");
    d.ws = a.ws;
    d.counters = a.counters;
  }
  static const bool no_bvec = getenv("RTENHIP_LAT_NO_BVEC") != nullptr;  // A/B experiments
  const bool pw = a.kh == 1 && a.kw == 1 && a.sh == 1 && a.sw == 1 && a.Hp == a.oh && a.Wp == a.ow;
  if (!no_bvec && v >= 70 && v < 90 && pw && d.P % 4 == 0 && d.x_img % 4 == 0 && d.kstride % 4 == 0 &&
      (uintptr_t)d.x % 16 == 0)
    d.bvec = 1;
  return RTENHIP_OK;
}

bool conv_lat_pair_ok(const ConvDmaArgs& a0, const ConvDmaArgs& a1) {
  const auto one = [](const ConvDmaArgs& a) {
    return a.groups == 1 && a.kh == 1 && a.kw == 1 && is_lat_cfg(a.cfg) && a.packed_w &&
           conv_dma_eligible(a.N, a.C, a.Hp, a.Wp, a.O, 1, a.C);
  };
  // a0 with 16-byte B copies (lat_conv_split_bvec's conditions)
  static const bool no_bvec = getenv("RTENHIP_LAT_NO_BVEC") != nullptr;
  const int64_t P = a0.oh * a0.ow;
  const bool bvec0 = !no_bvec && a0.sh == 1 && a0.sw == 1 && a0.Hp == a0.oh && a0.Wp == a0.ow && P % 4 == 0 &&
                     (a0.C * a0.Hp * a0.Wp) % 4 == 0 && (a0.Hp * a0.Wp) % 4 == 0 && (uintptr_t)a0.xin % 16 == 0;
  return bvec0 && one(a0) && one(a1) && lat_pair_variants_ok(a0.cfg - kLatCfgBase, a1.cfg - kLatCfgBase);
}

// Two ungrouped 1x1 latency convs in one launch (gemm_lat2_pair_kernel): a0
// must take 16-byte B copies (a pointwise stride-1 conv).
rtenhip_status conv_lat_pair(Ctx* c, const ConvDmaArgs& a0, const ConvDmaArgs& a1) {
  if (!conv_lat_pair_ok(a0, a1)) return fail(RTENHIP_UNSUPPORTED_VALUE, "latency conv pair: unsupported");
  const DmaTile tile{16, 256, 1};
  DmaDesc d0, d1;
  fill_conv_desc(a0, 0, true, tile, nullptr, d0);
  fill_conv_desc(a1, 0, true, tile, nullptr, d1);
  rtenhip_status st = lat_conv_split_bvec(a0, a0.cfg - kLatCfgBase, d0);
  if (!st) st = lat_conv_split_bvec(a1, a1.cfg - kLatCfgBase, d1);
  if (st) return st;
  if (!d0.bvec) return fail(RTENHIP_UNSUPPORTED_VALUE, "latency conv pair: first conv without 16-byte B copies");
  return launch_gemm_lat_pair(d0, a0.cfg - kLatCfgBase, d1, a1.cfg - kLatCfgBase, c->stream);
}

rtenhip_status conv_dma(Ctx* c, const ConvDmaArgs& a) {
  const int64_t opg = a.O / a.groups, ipg = a.C / a.groups;
  const int64_t K = ipg * a.kh * a.kw, P = a.oh * a.ow;
  const bool lat = is_lat_cfg(a.cfg);
  const int cfg = a.cfg >= 0 ? a.cfg : dma_default_cfg((int)opg, (int)(a.N * P), (int)K);
  const DmaTile tile = lat ? DmaTile{16, 256, 1} : dma_cfg_tile(cfg);
  // 1x1 kernels: koff(k) = k * Hp * Wp for any stride (no table needed by the
  // latency GEMM).
  const bool one_by_one = a.kh == 1 && a.kw == 1;
  const int* tab = nullptr;
  if (!(lat && one_by_one)) {
    tab = c->dtab((int)ipg, (int)a.Hp, (int)a.Wp, (int)a.kh, (int)a.kw, (int)a.dh, (int)a.dw);
    if (!tab) return fail(RTENHIP_HIP_ERROR, "DMA table allocation failed");
  }
  for (int64_t g = 0; g < a.groups; g++) {
    DmaDesc d;
    fill_conv_desc(a, g, lat, tile, tab, d);
    if (lat) {
      rtenhip_status st = lat_conv_split_bvec(a, cfg - kLatCfgBase, d);
      if (!st) st = launch_gemm_lat(d, cfg - kLatCfgBase, c->stream);
      if (st) return st;
      continue;
    }
    set_conv_bvec(a, cfg, tile, d);
    if (a.split) {
      const DmaSplit sp = dma_split_plan(d.M, d.N, d.K, cfg);
      if (sp.split_tiles > 0 && a.ws && a.counters && sp.ws_floats <= a.ws_cap && sp.counters <= a.cnt_cap) {
        d.split_tiles = sp.split_tiles;
        d.nkb = sp.nkb;
        d.ws = a.ws;
        d.counters = a.counters;
      }
    }
    d.persist_k = a.persist_k;
    rtenhip_status st = launch_gemm_dma(d, cfg, c->stream);
    if (st) return st;
  }
  return RTENHIP_OK;
}

// ResNet's conv3 + downsample pair as one dual DMA GEMM (gemm_dma_kernel
// DUAL): y = act((W3·h + b3) + (Wd·x + bd)), both ungrouped, same output.
// a3: conv3 (its residual is ignored: the downsample's value takes its
// place), ad: the downsample; both packed for cfg.
bool conv_dual_ok(const ConvDmaArgs& a3, const ConvDmaArgs& ad, int cfg) {
  return cfg >= 0 && cfg < dma_num_cfgs() && dma_cfg_dual(cfg) && a3.groups == 1 && ad.groups == 1 &&
         a3.O == ad.O && a3.N == ad.N && a3.oh == ad.oh && a3.ow == ad.ow && !a3.split &&
         conv_dma_eligible(a3.N, a3.C, a3.Hp, a3.Wp, a3.O, 1, a3.C * a3.kh * a3.kw) &&
         conv_dma_eligible(ad.N, ad.C, ad.Hp, ad.Wp, ad.O, 1, ad.C * ad.kh * ad.kw);
}

rtenhip_status conv_dma_dual(Ctx* c, const ConvDmaArgs& a3, const ConvDmaArgs& ad) {
  const int cfg = a3.cfg;
  if (!conv_dual_ok(a3, ad, cfg)) return fail(RTENHIP_UNSUPPORTED_VALUE, "conv pair not supported by the dual GEMM");
  const DmaTile tile = dma_cfg_tile(cfg);
  const int* t3 = c->dtab((int)a3.C, (int)a3.Hp, (int)a3.Wp, (int)a3.kh, (int)a3.kw, (int)a3.dh, (int)a3.dw);
  const int* td = c->dtab((int)ad.C, (int)ad.Hp, (int)ad.Wp, (int)ad.kh, (int)ad.kw, (int)ad.dh, (int)ad.dw);
  if (!t3 || !td) return fail(RTENHIP_HIP_ERROR, "DMA table allocation failed");
  DmaDesc d3, dd;
  fill_conv_desc(a3, 0, false, tile, t3, d3);
  fill_conv_desc(ad, 0, false, tile, td, dd);
  set_conv_bvec(a3, cfg, tile, d3);  // (kept only when both segments qualify, launch_gemm_dma)
  set_conv_bvec(ad, cfg, tile, dd);
  d3.residual = nullptr;
  d3.persist_k = a3.persist_k;
  return launch_gemm_dma(d3, cfg, c->stream, &dd);
}

const int2* Ctx::ktab(int C, int H, int W, int kh, int kw, int dh, int dw) {
  auto key = std::make_tuple(C, H, W, kh, kw, dh, dw);
  std::lock_guard<std::mutex> g(mu);
  auto it = ktabs.find(key);
  if (it != ktabs.end()) return it->second;
  // VirtualIm2Col row offsets (im2col.rs:104-124): row r = (c, ky, kx).
  std::vector<int2> tab((size_t)C * kh * kw);
  size_t r = 0;
  for (int c = 0; c < C; c++)
    for (int ky = 0; ky < kh; ky++)
      for (int kx = 0; kx < kw; kx++) {
        int kyd = ky * dh, kxd = kx * dw;
        tab[r].x = c * H * W + kyd * W + kxd;
        tab[r].y = (kyd << 16) | kxd;
        r++;
      }
  int2* d = nullptr;
  if (hipMalloc(&d, tab.size() * sizeof(int2)) != hipSuccess) return nullptr;
  if (hipMemcpy(d, tab.data(), tab.size() * sizeof(int2), hipMemcpyHostToDevice) != hipSuccess)
    return nullptr;
  ktabs[key] = d;
  return d;
}

// calc_output_size_and_padding (src/ops/pooling.rs:27-89).
rtenhip_status output_size_and_padding(int64_t in_h, int64_t in_w, int64_t k_h, int64_t k_w,
                                       int64_t stride_h, int64_t stride_w, int pad_mode,
                                       const int64_t* pads_in, int64_t dil_y, int64_t dil_x,
                                       int64_t out_hw[2], int64_t pads[4]) {
  if (dil_y == 0 || dil_x == 0) return fail(RTENHIP_INVALID_VALUE, "Dilations must be > 0");
  if (stride_h == 0 || stride_w == 0) return fail(RTENHIP_INVALID_VALUE, "Strides must be > 0");
  if (pad_mode == 1) {
    int64_t oh = (in_h + stride_h - 1) / stride_h, ow = (in_w + stride_w - 1) / stride_w;
    int64_t th = std::max<int64_t>(0, (oh - 1) * stride_h + (k_h - 1) * dil_y + 1 - in_h);
    int64_t tw = std::max<int64_t>(0, (ow - 1) * stride_w + (k_w - 1) * dil_x + 1 - in_w);
    pads[0] = th / 2;
    pads[1] = tw / 2;
    pads[2] = (th + 1) / 2;
    pads[3] = (tw + 1) / 2;
    out_hw[0] = oh;
    out_hw[1] = ow;
    return RTENHIP_OK;
  }
  if (!pads_in) return fail(RTENHIP_INVALID_VALUE, "Expected 4 padding values");
  for (int i = 0; i < 4; i++) pads[i] = pads_in[i];
  int64_t ph = in_h + pads[0] + pads[2], pw = in_w + pads[1] + pads[3];
  int64_t dkh = k_h + (k_h - 1) * (dil_y - 1), dkw = k_w + (k_w - 1) * (dil_x - 1);
  if (ph < dkh || pw < dkw) return fail(RTENHIP_INVALID_VALUE, "Input too small for kernel size");
  out_hw[0] = (ph - dil_y * (k_h - 1) - 1) / stride_h + 1;
  out_hw[1] = (pw - dil_x * (k_w - 1) - 1) / stride_w + 1;
  return RTENHIP_OK;
}

static bool g_split_enabled = true;

rtenhip_status plan_conv(const rtenhip_tensor* x, const rtenhip_tensor* w, int pad_mode,
                                const int64_t* pads, const int64_t* strides,
                                const int64_t* dilations, int64_t groups, ConvPlan& p) {
  if (!x || !w) return fail(RTENHIP_MISSING_INPUTS, "Missing inputs");
  p.one_d = x->ndim == 3;
  int64_t p4[4] = {0, 0, 0, 0};
  if (p.one_d) {
    // conv.rs:96-143: 1-D conv as 2-D with H = 1.
    if (w->ndim != 3) return fail(RTENHIP_INVALID_VALUE, "Expected kernel to have 3 dims");
    p.N = x->shape[0];
    p.C = x->shape[1];
    p.H = 1;
    p.W = x->shape[2];
    p.O = w->shape[0];
    p.KC = w->shape[1];
    p.kh = 1;
    p.kw = w->shape[2];
    p.sh = 1;
    p.sw = strides ? strides[0] : 1;
    p.dh = 1;
    p.dw = dilations ? dilations[0] : 1;
    if (pads) {
      p4[1] = pads[0];
      p4[3] = pads[1];
    }
  } else {
    if (x->ndim != 4) return fail(RTENHIP_INVALID_VALUE, "Expected input to have 4 dims");
    if (w->ndim != 4) return fail(RTENHIP_INVALID_VALUE, "Expected kernel to have 4 dims");
    p.N = x->shape[0];
    p.C = x->shape[1];
    p.H = x->shape[2];
    p.W = x->shape[3];
    p.O = w->shape[0];
    p.KC = w->shape[1];
    p.kh = w->shape[2];
    p.kw = w->shape[3];
    p.sh = strides ? strides[0] : 1;
    p.sw = strides ? strides[1] : 1;
    p.dh = dilations ? dilations[0] : 1;
    p.dw = dilations ? dilations[1] : 1;
    if (pads)
      for (int i = 0; i < 4; i++) p4[i] = pads[i];
  }
  p.groups = groups;
  int64_t ohw[2];
  rtenhip_status st = output_size_and_padding(p.H, p.W, p.kh, p.kw, p.sh, p.sw, pad_mode, p4, p.dh,
                                              p.dw, ohw, p.pads);
  if (st) return st;
  p.oh = ohw[0];
  p.ow = ohw[1];
  if (groups == 0 || p.C / groups != p.KC)
    return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES,
                "Input channels (per group) does not match kernel input channels");
  if (p.C % groups != 0 || p.O % groups != 0)
    return fail(RTENHIP_INCOMPATIBLE_INPUT_SHAPES,
                "Input channels and output channels must be divisible by group count");
  return RTENHIP_OK;
}

bool conv_takes_dma(const ConvPlan& p) {
  const bool has_pad = p.pads[0] || p.pads[1] || p.pads[2] || p.pads[3];
  const bool pointwise = p.kh == 1 && p.kw == 1 && !has_pad && p.groups == 1 && p.sh == 1 &&
                         p.sw == 1 && p.dh == 1 && p.dw == 1;
  const bool depthwise = p.C == p.O && p.groups == p.C;
  const int64_t Hp = p.H + p.pads[0] + p.pads[2], Wp = p.W + p.pads[1] + p.pads[3];
  return !depthwise && !(pointwise && p.O == 1) && p.N * p.oh * p.ow > 0 &&
         conv_dma_eligible(p.N, p.C, Hp, Wp, p.O, p.groups, (p.C / p.groups) * p.kh * p.kw);
}

rtenhip_status pack_conv_weights(Ctx* c, const float* w, const ConvPlan& p, int cfg, float* out) {
  const int64_t opg = p.O / p.groups, K = (p.C / p.groups) * p.kh * p.kw;
  if (is_lat_cfg(cfg)) {
    const int64_t per = lat_packed_floats((int)opg, (int)K);
    for (int64_t g = 0; g < p.groups; g++) {
      rtenhip_status st = launch_pack_lat(w + g * opg * K, K, (int)opg, (int)K, out + g * per, c->stream);
      if (st) return st;
    }
    return RTENHIP_OK;
  }
  const DmaTile tile = dma_cfg_tile(cfg);
  const int64_t per_group = packed_a_floats((int)opg, (int)K, tile);
  for (int64_t g = 0; g < p.groups; g++) {
    rtenhip_status st =
        launch_pack_a(w + g * opg * K, K, (int)opg, (int)K, tile, out + g * per_group, c->stream);
    if (st) return st;
  }
  return RTENHIP_OK;
}

int64_t packed_conv_weight_floats(const ConvPlan& p, int cfg) {
  const int64_t opg = p.O / p.groups, K = (p.C / p.groups) * p.kh * p.kw;
  if (is_lat_cfg(cfg)) return lat_packed_floats((int)opg, (int)K) * p.groups;
  return packed_a_floats((int)opg, (int)K, dma_cfg_tile(cfg)) * p.groups;
}

rtenhip_status conv_impl(Ctx* c, const rtenhip_tensor* x, const rtenhip_tensor* w,
                         const float* bias, int pad_mode, const int64_t* pads,
                         const int64_t* strides, const int64_t* dilations, int64_t groups,
                         const float* residual, int act, float lo, float hi, rtenhip_tensor* y) {
  ConvPlan p;
  rtenhip_status st = plan_conv(x, w, pad_mode, pads, strides, dilations, groups, p);
  if (st) return st;
  hipStream_t s = c->stream;
  if (!is_contiguous(*w)) return fail(RTENHIP_UNSUPPORTED_VALUE, "Conv weights must be contiguous");
  const float* xd = x->data;
  if (!is_contiguous(*x)) {
    float* tmp = c->scratch_floats(numel(*x), 0);
    if (!tmp) return fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
    st = launch_copy_strided(*x, tmp, s);
    if (st) return st;
    xd = tmp;
  }
  const int64_t P = p.oh * p.ow;
  const bool has_pad = p.pads[0] || p.pads[1] || p.pads[2] || p.pads[3];
  if (p.N == 0 || p.O == 0 || P == 0) return RTENHIP_OK;

  const int64_t Hp = p.H + p.pads[0] + p.pads[2], Wp = p.W + p.pads[1] + p.pads[3];
  if (c->use_dma && conv_takes_dma(p)) {
    // Fast path: zero-bordered input + packed weights + LDS-DMA GEMM.
    const float* xin = xd;
    if (has_pad) {
      float* xp = c->scratch_floats((size_t)(p.N * p.C * Hp * Wp), 1);
      if (!xp) return fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
      st = launch_pad_nchw(xd, xp, p.N * p.C, (int)p.H, (int)p.W, (int)p.pads[0], (int)p.pads[1],
                           (int)p.pads[2], (int)p.pads[3], s);
      if (st) return st;
      xin = xp;
    }
    const int64_t opg = p.O / p.groups, K = (p.C / p.groups) * p.kh * p.kw;
    const int cfg = dma_default_cfg((int)opg, (int)(p.N * P), (int)K);
    const DmaTile tile = dma_cfg_tile(cfg);
    const int64_t per_group = packed_a_floats((int)opg, (int)K, tile);
    float* wp = nullptr;
    auto key = std::make_tuple((const void*)w->data, opg * p.groups, K, tile.bm, tile.bk, tile.il);
    if (c->trust_weight_cache) {
      auto it = c->packed_cache.find(key);
      if (it != c->packed_cache.end()) wp = it->second;
    }
    if (!wp) {
      if (c->trust_weight_cache) {
        if (hipMalloc(&wp, (size_t)(per_group * p.groups) * 4) != hipSuccess)
          return fail(RTENHIP_HIP_ERROR, "hipMalloc failed");
        c->packed_cache[key] = wp;
      } else {
        wp = c->scratch_floats((size_t)(per_group * p.groups), 2);
        if (!wp) return fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
      }
      for (int64_t g = 0; g < p.groups; g++) {
        st = launch_pack_a(w->data + g * opg * K, K, (int)opg, (int)K, tile, wp + g * per_group, s);
        if (st) return st;
      }
    }
    ConvDmaArgs a{};
    a.xin = xin;
    a.N = p.N;
    a.C = p.C;
    a.Hp = Hp;
    a.Wp = Wp;
    a.O = p.O;
    a.kh = p.kh;
    a.kw = p.kw;
    a.sh = p.sh;
    a.sw = p.sw;
    a.dh = p.dh;
    a.dw = p.dw;
    a.oh = p.oh;
    a.ow = p.ow;
    a.groups = p.groups;
    a.packed_w = wp;
    a.bias = bias;
    a.residual = residual;
    a.act = act;
    a.lo = lo;
    a.hi = hi;
    a.y = y->data;
    a.y_img = p.O * P;
    a.cfg = cfg;
    if (g_split_enabled) {
      const DmaSplit sp = dma_split_plan((int)opg, (int)(p.N * P), (int)K, cfg);
      if (sp.split_tiles > 0) {
        a.ws = c->scratch_floats((size_t)sp.ws_floats, 3);
        a.counters = c->split_counters((size_t)sp.counters);
        if (!a.ws || !a.counters) return fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
        a.split = true;
        a.ws_cap = sp.ws_floats;
        a.cnt_cap = sp.counters;
      }
    }
    return conv_dma(c, a);
  }

  if (p.kh == 1 && p.kw == 1 && !has_pad && p.groups == 1 && p.sh == 1 && p.sw == 1 &&
      p.dh == 1 && p.dw == 1) {
    // conv_2d_pointwise (conv.rs:24-68): per image W[O,C] @ X_n[C,HW] (+bias).
    if (p.O == 1) {
      // A has one row -> the reference takes gemv (gemm.rs:767-780).
      for (int64_t n = 0; n < p.N; n++) {
        st = launch_gemv(P, p.C, w->data, xd + n * p.C * P, P, 1, y->data + n * P, 1.f, 0.f, bias,
                         c->ref_threads, s);
        if (st) return st;
      }
      if (residual || act) {
        // Rare path: apply fused epilogue as separate elementwise passes.
        if (residual) {
          BcastDesc d{};
          st = launch_binary(RTENHIP_BINARY_ADD, y->data, residual, y->data, p.N * P, d, 0, 1, 1, s);
          if (st) return st;
        }
        if (act == RTENHIP_ACT_RELU) st = launch_unary(RTENHIP_UNARY_RELU, y->data, y->data, p.N * P, 0, 0, s);
        if (act == RTENHIP_ACT_CLIP) st = launch_unary(RTENHIP_UNARY_CLIP, y->data, y->data, p.N * P, lo, hi, s);
      }
      return st;
    }
    GemmDesc d{};
    d.M = (int)p.O;
    d.N = (int)(p.N * P);
    d.K = (int)p.C;
    d.a = w->data;
    d.a_m = p.C;
    d.a_k = 1;
    d.bmode = 2;
    d.b = xd;
    d.C = (int)p.C;
    d.H = (int)p.H;
    d.W = (int)p.W;
    d.OW = (int)p.ow;
    d.P = (int)P;
    d.x_img = p.C * p.H * p.W;
    d.omode = 1;
    d.out = y->data;
    d.out_img = p.O * P;
    d.bias = bias;
    d.residual = residual;
    d.alpha = 1.f;
    d.beta = 0.f;
    d.act = act;
    d.act_lo = lo;
    d.act_hi = hi;
    return launch_gemm(d, s);
  }
  if (p.C == p.O && p.groups == p.C) {
    return launch_depthwise(xd, w->data, bias, y->data, (int)p.N, (int)p.C, (int)p.H, (int)p.W,
                            (int)p.oh, (int)p.ow, (int)p.kh, (int)p.kw, (int)p.sh, (int)p.sw,
                            (int)p.dh, (int)p.dw, (int)p.pads[0], (int)p.pads[1], residual, act,
                            lo, hi, s);
  }
  const int64_t opg = p.O / p.groups, ipg = p.C / p.groups;
  const int64_t K = ipg * p.kh * p.kw;
  const int2* tab = c->ktab((int)ipg, (int)p.H, (int)p.W, (int)p.kh, (int)p.kw, (int)p.dh,
                            (int)p.dw);
  if (!tab) return fail(RTENHIP_HIP_ERROR, "im2col table allocation failed");
  for (int64_t g = 0; g < p.groups; g++) {
    GemmDesc d{};
    d.M = (int)opg;
    d.N = (int)(p.N * P);
    d.K = (int)K;
    d.a = w->data + g * opg * K;
    d.a_m = K;
    d.a_k = 1;
    d.bmode = 1;
    d.b = xd + g * ipg * p.H * p.W;
    d.C = (int)ipg;
    d.H = (int)p.H;
    d.W = (int)p.W;
    d.OW = (int)p.ow;
    d.P = (int)P;
    d.sh = (int)p.sh;
    d.sw = (int)p.sw;
    d.pt = (int)p.pads[0];
    d.pl = (int)p.pads[1];
    d.x_img = p.C * p.H * p.W;
    d.ktab = tab;
    d.omode = 1;
    d.out = y->data + g * opg * P;
    d.out_img = p.O * P;
    d.bias = bias ? bias + g * opg : nullptr;
    d.residual = residual ? residual + g * opg * P : nullptr;
    d.alpha = 1.f;
    d.beta = 0.f;
    d.act = act;
    d.act_lo = lo;
    d.act_hi = hi;
    st = launch_gemm(d, s);
    if (st) return st;
  }
  return RTENHIP_OK;
}

bool dense_dma_eligible(int64_t M, int64_t N, int64_t K, int64_t a_cs, int64_t b_rs, int64_t b_cs) {
  // Large enough for MFMA tiles to pay for the per-call A pack; N % 4 == 0 for
  // 16-byte B copies and epilogue stores; B addressed with 32-bit offsets.
  return M >= 128 && N >= 128 && K >= 16 && N % 4 == 0 && a_cs == 1 && b_cs == 1 &&
         b_rs % 4 == 0 && b_rs >= N && M * N * K >= (int64_t(1) << 24) &&
         K * b_rs < (int64_t(1) << 29) && M < (int64_t(1) << 30);
}

static bool dense_vec4(const DenseDmaArgs& a) {
  return a.out_rs % 4 == 0 && (uintptr_t)a.out % 16 == 0 &&
         (!a.residual || (a.res_rs % 4 == 0 && (uintptr_t)a.residual % 16 == 0)) &&
         (!a.colbias || (uintptr_t)a.colbias % 16 == 0);
}

bool dense_dma_pk_out_ok(const DenseDmaArgs& a, int cfg) {
  const DmaTile& t = a.pk_tile;
  auto pow2 = [](int v) { return v > 0 && (v & (v - 1)) == 0; };
  return cfg >= 0 && cfg < dma_num_cfgs() && dense_vec4(a) && dma_cfg_vec_epilogue(cfg) && a.N % 4 == 0 &&
         a.pk_K == a.N && pow2(t.bm) && pow2(t.bk) && t.bk >= 8 && t.bm >= 32;
}

rtenhip_status gemm_dense_dma(Ctx* c, const DenseDmaArgs& a) {
  hipStream_t s = c->stream;
  const int cfg = a.cfg >= 0 ? a.cfg : dma_default_cfg((int)a.M, (int)a.N, (int)a.K);
  const DmaTile tile = dma_cfg_tile(cfg);
  float* pk = a.pk;
  if (!pk) {
    pk = c->scratch_floats((size_t)packed_a_floats((int)a.M, (int)a.K, tile), 2);
    if (!pk) return fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
  }
  if (a.pack || !a.pk) {
    rtenhip_status st = launch_pack_a(a.a, a.a_rs, (int)a.M, (int)a.K, tile, pk, s);
    if (st) return st;
  }
  // B as a one-image pointwise conv input [1, C = K, H = 1, W = b_rs].
  const int* tab = c->dtab((int)a.K, 1, (int)a.b_rs, 1, 1, 1, 1);
  if (!tab) return fail(RTENHIP_HIP_ERROR, "DMA table allocation failed");
  DmaDesc d{};
  d.M = (int)a.M;
  d.N = (int)a.N;
  d.K = (int)a.K;
  d.tile = tile;
  d.apk = pk;
  // Segments (DenseDmaArgs::n_seg) are the GEMM's "images": B, the output
  // and the residual step by one segment per image.
  const int64_t nseg = a.n_seg > 1 ? a.n_seg : 1;
  if (a.N % nseg || (nseg > 1 && (a.residual || a.pk_out)))
    return fail(RTENHIP_INVALID_VALUE, "segmented dense GEMM: unsupported operands");
  const int64_t segn = a.N / nseg;
  // The kernel addresses B and the output segments with 32-bit byte offsets.
  if (nseg > 1 && (uint64_t)nseg * a.K * a.b_rs * 4 >= (1ull << 32))
    return fail(RTENHIP_UNSUPPORTED_VALUE, "segmented dense GEMM: operands exceed 32-bit offsets");
  d.x = a.b;
  d.x_bytes = (uint32_t)(nseg * a.K * a.b_rs * 4);
  d.x_img = a.K * a.b_rs;
  d.ystride = 0;
  d.xstride = 1;
  d.OW = (int)segn;
  d.P = (int)segn;
  d.fdOW = make_fastdiv((uint32_t)segn);
  d.fdP = make_fastdiv((uint32_t)segn);
  d.ktab4 = tab;
  d.out = a.out;
  d.out_img = a.M * a.out_rs;
  d.out_c = a.out_rs;
  d.out_row = a.N;
  d.out_off = 0;
  d.residual = a.residual;
  d.res_img = a.M * a.res_rs;
  d.res_c = a.res_rs;
  d.bias = a.bias;
  d.colbias = a.colbias;
  d.alpha = 1.f;
  d.beta = 0.f;
  d.act = a.act;
  d.act_lo = a.lo;
  d.act_hi = a.hi;
  // 16-byte epilogue: rows contiguous in memory segments of 4.
  d.vec4 = dense_vec4(a) ? 1 : 0;
  if (a.pk_out) {
    if (!dense_dma_pk_out_ok(a, cfg)) return fail(RTENHIP_INVALID_VALUE, "packed-A output not possible here");
    d.pk_out = a.pk_out;
    d.pk_lbm = __builtin_ctz(a.pk_tile.bm);
    d.pk_lbk = __builtin_ctz(a.pk_tile.bk);
    d.pk_tiles_k = (int)((a.pk_K + a.pk_tile.bk - 1) / a.pk_tile.bk);
  }
  if (dma_cfg_bvec(cfg) && a.K % tile.bk == 0 && ((uintptr_t)a.b % 16) == 0) {
    d.bvec = 1;
    d.kstride = (int)a.b_rs;
  }
  if (a.split) {
    const DmaSplit sp = dma_split_plan(d.M, d.N, d.K, cfg);
    if (sp.split_tiles > 0) {
      float* ws = a.ws;
      int* cnt = a.counters;
      if (!ws || sp.ws_floats > a.ws_cap || !cnt || sp.counters > a.cnt_cap) {
        ws = c->scratch_floats((size_t)sp.ws_floats, 3);
        cnt = c->split_counters((size_t)sp.counters);
        if (!ws || !cnt) return fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
      }
      d.split_tiles = sp.split_tiles;
      d.nkb = sp.nkb;
      d.ws = ws;
      d.counters = cnt;
    }
  }
  d.persist_k = a.persist_k;
  d.swz = dma_dense_swz(a.K, dma_cfg_info_bn(cfg));  // strip tile order (dense MatMuls only)
  return launch_gemm_dma(d, cfg, s);
}

// GemmExecutor::gemm_bias on strided device matrices (gemm.rs:733-930).
rtenhip_status gemm_impl(Ctx* c, int64_t m, int64_t n, int64_t k, const float* a, int64_t a_rs,
                         int64_t a_cs, const float* b, int64_t b_rs, int64_t b_cs, float* out,
                         int64_t out_rs, float alpha, float beta, const float* bias, int act) {
  hipStream_t s = c->stream;
  if (m == 0 || n == 0) return RTENHIP_OK;
  if (m == 1 && k > 0 && act == 0) {
    return launch_gemv(n, k, a, b, b_rs, b_cs, out, alpha, beta, bias, c->ref_threads, s);
  }
  GemmDesc d{};
  d.M = (int)m;
  d.N = (int)n;
  d.K = (int)k;
  d.a = a;
  d.a_m = a_rs;
  d.a_k = a_cs;
  d.bmode = 0;
  d.b = b;
  d.b_k = b_rs;
  d.b_n = b_cs;
  d.omode = 0;
  d.out = out;
  d.out_m = out_rs;
  d.bias = bias;
  d.cin = beta != 0.f ? out : nullptr;
  d.alpha = alpha;
  d.beta = beta;
  d.act = act;
  if (k == 0) {
    // gemm.rs:757-765: out = beta * (beta == 0 ? 0 : out), no bias.
    d.a = nullptr;
    d.bias = nullptr;
  }
  if (gemm_smallm_eligible(d)) {
    float* ws = c->scratch_floats((size_t)gemm_smallm_ws_floats(d), 3);
    if (!ws) return fail(RTENHIP_HIP_ERROR, "scratch allocation failed");
    return launch_gemm_smallm(d, ws, s);
  }
  if (c->use_dma && k > 0 && alpha == 1.f && beta == 0.f && out_rs == n &&
      dense_dma_eligible(m, n, k, a_cs, b_rs, b_cs) && gemm_forced_cfg() < 0) {
    DenseDmaArgs da{};
    da.M = m;
    da.N = n;
    da.K = k;
    da.a = a;
    da.a_rs = a_rs;
    da.b = b;
    da.b_rs = b_rs;
    da.out = out;
    da.out_rs = out_rs;
    da.bias = bias;
    da.act = act;
    da.cfg = -1;
    da.split = g_split_enabled;
    return gemm_dense_dma(c, da);
  }
  return launch_gemm(d, s);
}

}  // namespace rtenhip

using namespace rtenhip;

static Ctx* C_(rtenhip_ctx* c) { return reinterpret_cast<Ctx*>(c); }

extern "C" {

rtenhip_ctx* rtenhip_create(int device) {
  if (hipSetDevice(device) != hipSuccess) {
    set_error(RTENHIP_HIP_ERROR, "hipSetDevice failed");
    return nullptr;
  }
  return reinterpret_cast<rtenhip_ctx*>(new Ctx(device));
}

void rtenhip_destroy(rtenhip_ctx* ctx) { delete C_(ctx); }

rtenhip_status rtenhip_set_stream(rtenhip_ctx* ctx, void* stream) {
  C_(ctx)->stream = reinterpret_cast<hipStream_t>(stream);
  return RTENHIP_OK;
}
void* rtenhip_get_stream(rtenhip_ctx* ctx) { return C_(ctx)->stream; }

rtenhip_status rtenhip_set_exec_stream(rtenhip_ctx* ctx, void* stream) {
  Ctx* c = C_(ctx);
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (s == c->exec_stream) return RTENHIP_OK;
  if (c->exec_stream) RTENHIP_HIP_CHECK(hipStreamSynchronize(c->exec_stream));
  if (c->exec_stream && c->owns_exec) (void)hipStreamDestroy(c->exec_stream);
  c->exec_stream = s;  // NULL: the next graph run creates a library-owned one
  c->owns_exec = false;
  return RTENHIP_OK;
}

const char* rtenhip_last_error_message(void) { return g_err.c_str(); }
int32_t rtenhip_last_error_code(void) { return g_err_code; }

rtenhip_status rtenhip_synchronize(rtenhip_ctx* ctx) {
  RTENHIP_HIP_CHECK(hipStreamSynchronize(C_(ctx)->stream));
  return RTENHIP_OK;
}

void* rtenhip_malloc(rtenhip_ctx*, size_t bytes) {
  void* p = nullptr;
  if (hipMalloc(&p, bytes ? bytes : 4) != hipSuccess) return nullptr;
  return p;
}
void rtenhip_free(rtenhip_ctx*, void* ptr) {
  if (ptr) (void)hipFree(ptr);
}
rtenhip_status rtenhip_memcpy_h2d(rtenhip_ctx* ctx, void* dst, const void* src, size_t bytes) {
  RTENHIP_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, C_(ctx)->stream));
  RTENHIP_HIP_CHECK(hipStreamSynchronize(C_(ctx)->stream));
  return RTENHIP_OK;
}
rtenhip_status rtenhip_memcpy_d2h(rtenhip_ctx* ctx, void* dst, const void* src, size_t bytes) {
  RTENHIP_HIP_CHECK(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, C_(ctx)->stream));
  RTENHIP_HIP_CHECK(hipStreamSynchronize(C_(ctx)->stream));
  return RTENHIP_OK;
}

int32_t rtenhip_num_threads(rtenhip_ctx* ctx) { return C_(ctx)->ref_threads; }
void rtenhip_cpu_counts(int32_t* logical, int32_t* physical) {
  if (logical) *logical = logical_cpus();
  if (physical) *physical = physical_cpus();
}

const char* rtenhip_build_info(void) { return "rten-hip gfx950 (CDNA4) f32 MFMA backend v0.1"; }

// Tuning / test knob: route convs through the LDS-DMA GEMM (default) or the
// register-staged general kernel.  Both produce bit-identical results.
void rtenhip_debug_set_dma(rtenhip_ctx* ctx, int enabled) { C_(ctx)->use_dma = enabled != 0; }
void rtenhip_debug_set_split(int enabled) { rtenhip::g_split_enabled = enabled != 0; }
void rtenhip_debug_trust_weight_cache(rtenhip_ctx* ctx, int enabled) {
  C_(ctx)->trust_weight_cache = enabled != 0;
}

rtenhip_status rtenhip_output_size_and_padding(int64_t in_h, int64_t in_w, int64_t k_h,
                                               int64_t k_w, int64_t stride_h, int64_t stride_w,
                                               int pad_mode, const int64_t pads_in[4],
                                               int64_t dil_h, int64_t dil_w, int64_t out_hw[2],
                                               int64_t pads_out[4]) {
  return output_size_and_padding(in_h, in_w, k_h, k_w, stride_h, stride_w, pad_mode, pads_in,
                                 dil_h, dil_w, out_hw, pads_out);
}

rtenhip_status rtenhip_gemm_f32(rtenhip_ctx* ctx, int64_t m, int64_t n, int64_t k,
                                const float* a, int64_t a_rs, int64_t a_cs, const float* b,
                                int64_t b_rs, int64_t b_cs, float* out, int64_t out_rs,
                                float alpha, float beta, const float* bias) {
  return gemm_impl(C_(ctx), m, n, k, a, a_rs, a_cs, b, b_rs, b_cs, out, out_rs, alpha, beta, bias,
                   0);
}

rtenhip_status rtenhip_conv_output_shape(const rtenhip_tensor* x, const rtenhip_tensor* w,
                                         int pad_mode, const int64_t* pads,
                                         const int64_t* strides, const int64_t* dilations,
                                         int64_t groups, int64_t* out_shape, int32_t* out_ndim) {
  ConvPlan p;
  rtenhip_status st = plan_conv(x, w, pad_mode, pads, strides, dilations, groups, p);
  if (st) return st;
  out_shape[0] = p.N;
  out_shape[1] = p.O;
  if (p.one_d) {
    out_shape[2] = p.ow;
    *out_ndim = 3;
  } else {
    out_shape[2] = p.oh;
    out_shape[3] = p.ow;
    *out_ndim = 4;
  }
  return RTENHIP_OK;
}

rtenhip_status rtenhip_conv_f32(rtenhip_ctx* ctx, const rtenhip_tensor* x,
                                const rtenhip_tensor* w, const float* bias, int pad_mode,
                                const int64_t* pads, const int64_t* strides,
                                const int64_t* dilations, int64_t groups, const float* residual,
                                int act, float act_lo, float act_hi, rtenhip_tensor* y) {
  int64_t os[4];
  int32_t ond;
  rtenhip_status st =
      rtenhip_conv_output_shape(x, w, pad_mode, pads, strides, dilations, groups, os, &ond);
  if (st) return st;
  if (!y || y->ndim != ond) return fail(RTENHIP_INCORRECT_OUTPUT_TYPE, "Output has wrong rank");
  for (int i = 0; i < ond; i++)
    if (y->shape[i] != os[i]) return fail(RTENHIP_INCORRECT_OUTPUT_TYPE, "Output has wrong shape");
  if (!is_contiguous(*y)) return fail(RTENHIP_UNSUPPORTED_VALUE, "Output must be contiguous");
  return conv_impl(C_(ctx), x, w, bias, pad_mode, pads, strides, dilations, groups, residual, act,
                   act_lo, act_hi, y);
}

}  // extern "C"
