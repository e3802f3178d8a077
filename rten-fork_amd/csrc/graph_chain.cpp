// Conv chains of a plan (Plan::ConvChain, conv_chain.hip): which runs of
// convs become one persistent launch, their layer / phase tables, and the
// build-time check that the chain beats the convs launched one by one.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <set>
#include <string>
#include <vector>

#include "chain.h"
#include "graph.h"

namespace rtenhip {

namespace {

struct Range {
  uintptr_t lo = 0, hi = 0;
  bool overlaps(const Range& o) const { return lo < hi && o.lo < o.hi && lo < o.hi && o.lo < hi; }
};

Range range_of(const void* p, int64_t floats) {
  Range r;
  if (p && floats > 0) {
    r.lo = (uintptr_t)p;
    r.hi = r.lo + (uintptr_t)floats * 4;
  }
  return r;
}

}  // namespace

// Chains are cut from the plan's op order: maximal runs of consecutive convs
// that (a) the plan runs on the DMA / latency GEMM (ungrouped 1x1 or 3x3
// kernels, not an FC layer, not part of a MobileNetV2 fusion or a broadcast
// residual); (b) read an unpadded input or one their producer zero-borders;
// (c) touch no graph input or output (the tables hold plan-fixed pointers).
// A run becomes a chain when at least half of its convs were tuned to the
// latency GEMM (small batches) or RTENHIP_CHAIN=1, and is kept when one launch
// of it times faster than its convs one by one (RTENHIP_CHAIN=1 keeps it
// regardless).  Values the chain both produces and consumes (and that are not
// zero-bordered, which have storage of their own already) get chain-owned
// buffers, so no storage is reused inside the launch; an output that leaves
// the chain keeps its arena slot, which must not overlap anything used in
// its phase or later (checked; the run is not chained otherwise).
rtenhip_status Graph::build_chains(Plan& p) {
  for (auto& c : p.chains) c.release();
  p.chains.clear();
  p.chain_of.clear();
  p.chains_built = true;
  p.chains_arena = arena;
  if (chain_mode == 0 || !ctx->use_dma) return RTENHIP_OK;
  std::set<int> io(p.input_ids.begin(), p.input_ids.end());
  io.insert(p.output_ids.begin(), p.output_ids.end());
  auto eligible = [&](int op) {
    auto it = p.convs.find(op);
    if (it == p.convs.end()) return false;
    const ConvExec& ce = it->second;
    const ConvPlan& g = ce.g;
    if (ce.fc || g.groups != 1 || g.one_d) return false;
    if (!((g.kh == 1 && g.kw == 1) || (g.kh == 3 && g.kw == 3))) return false;
    if (p.expand_fused.count(op) || p.dwpw_fused.count(op) || p.conv_unfused.count(op) || p.conv_pair.count(op) ||
        p.pair_hold.count(op))
      return false;
    const Node& n = nodes[op];
    const bool has_pad = g.pads[0] || g.pads[1] || g.pads[2] || g.pads[3];
    if (has_pad && !p.padded.count(n.inputs[0])) return false;
    for (int v : {n.inputs[0], n.fused_residual, n.outputs[0]})
      if (v >= 0 && io.count(v)) return false;
    return true;
  };
  std::vector<std::vector<int>> runs;
  std::vector<int> cur;
  for (int op : p.ops) {
    if (eligible(op)) {
      cur.push_back(op);
    } else {
      if (cur.size() >= 2) runs.push_back(cur);
      cur.clear();
    }
  }
  if (cur.size() >= 2) runs.push_back(cur);
  if (runs.empty()) return RTENHIP_OK;

  hipStream_t s = ctx->stream;
  std::map<int, std::vector<int>> consumers;  // value -> plan ops reading it
  for (int op : p.ops) {
    const Node& n = nodes[op];
    for (int v : n.inputs)
      if (v >= 0) consumers[v].push_back(op);
    if (n.fused_residual >= 0) consumers[n.fused_residual].push_back(op);
  }
  for (const std::vector<int>& run : runs) {
    int lat = 0;
    for (int op : run) lat += is_lat_cfg(p.convs[op].cfg) ? 1 : 0;
    // Auto mode: long runs only (a launch saved per conv is what the chain
    // can win; a short run cannot repay its barriers).
    if (chain_mode != 1 && (2 * lat < (int)run.size() || run.size() < 8)) continue;
    Plan::ConvChain c;
    c.ops = run;
    const std::set<int> in_run(run.begin(), run.end());
    std::map<int, int> producer;  // value -> layer index (run order)
    for (size_t i = 0; i < run.size(); i++) producer[nodes[run[i]].outputs[0]] = (int)i;
    rtenhip_status st = RTENHIP_OK;
    auto alloc = [&](size_t bytes, bool zero) -> void* {
      void* b = nullptr;
      if (hipMalloc(&b, bytes) != hipSuccess) return nullptr;
      c.owned.push_back(b);
      if (zero && hipMemsetAsync(b, 0, bytes, s) != hipSuccess) return nullptr;
      return b;
    };
    std::map<int, float*> priv;
    for (int op : run) {
      const int v = nodes[op].outputs[0];
      if (p.padded.count(v)) continue;
      bool inside = consumers.count(v) > 0;
      for (int cop : consumers[v]) inside = inside && in_run.count(cop) > 0;
      if (!inside) continue;
      const ConvPlan& g = p.convs[op].g;
      float* b = static_cast<float*>(alloc((size_t)(g.N * g.O * g.oh * g.ow) * 4, false));
      if (!b) {
        st = fail(RTENHIP_HIP_ERROR, "conv chain: hipMalloc failed");
        break;
      }
      priv[v] = b;
    }
    const int nl = (int)run.size();
    std::vector<ChainLayer> layers(nl);
    std::vector<int> phase(nl, 0);
    std::vector<Range> in_r(nl), res_r(nl), out_r(nl);
    std::vector<bool> arena_out(nl, false);
    for (int L = 0; !st && L < nl; L++) {
      const int op = run[L];
      const Node& n = nodes[op];
      ConvExec& ce = p.convs[op];
      const ConvPlan& g = ce.g;
      ConvDmaArgs a{};
      conv_io_args(p, op, a);
      if (priv.count(n.inputs[0]) && !p.padded.count(n.inputs[0])) a.xin = priv[n.inputs[0]];
      if (n.fused_residual >= 0 && priv.count(n.fused_residual)) a.residual = priv[n.fused_residual];
      if (priv.count(n.outputs[0])) {
        a.y = priv[n.outputs[0]];
        a.y_img = g.O * g.oh * g.ow;
        a.y_row = a.y_off = 0;
      } else if (!p.padded.count(n.outputs[0])) {
        arena_out[L] = true;
      }
      const int v = ce.cfg - kLatCfgBase;
      const int rw = (is_lat_cfg(ce.cfg) && v >= 71 && v <= 74 && v != 73) ? v - 70 : 2;
      if (is_lat_cfg(ce.cfg) && ce.packed) {
        a.packed_w = ce.packed;  // lat-packed ([sub][kb][group][lane], the same for every variant)
      } else {
        float* pk = static_cast<float*>(alloc((size_t)packed_conv_weight_floats(g, kLatCfgBase + 72) * 4, false));
        if (!pk) {
          st = fail(RTENHIP_HIP_ERROR, "conv chain: hipMalloc failed");
          break;
        }
        if ((st = pack_conv_weights(ctx, ptr_of(p, n.inputs[1]), g, kLatCfgBase + 72, pk))) break;
        a.packed_w = pk;
      }
      ChainLayer& ly = layers[L];
      if ((st = lat_conv_desc(a, ly.d))) break;
      ly.rw = rw;
      ly.cw = 4 / rw;
      {
        static const bool no_bvec = getenv("RTENHIP_CHAIN_NO_BVEC") != nullptr;  // A/B experiments
        const bool pw = g.kh == 1 && g.kw == 1 && g.sh == 1 && g.sw == 1 && a.Hp == g.oh && a.Wp == g.ow;
        ly.bvec = (!no_bvec && pw && ly.d.P % 4 == 0 && ly.d.x_img % 4 == 0 && ly.d.kstride % 4 == 0 &&
                   (uintptr_t)ly.d.x % 16 == 0)
                      ? 1
                      : 0;
      }
      ly.subs = (ly.d.M + 15) / 16;
      ly.wg_m = (ly.subs + rw - 1) / rw;
      ly.wg_n = ((ly.d.N + 15) / 16 + ly.cw - 1) / ly.cw;
      ly.nkb = (ly.d.K + 255) / 256;
      const int64_t items = (int64_t)ly.wg_m * ly.wg_n * ly.nkb;
      if (items > (1 << 28)) {
        st = fail(RTENHIP_UNSUPPORTED_VALUE, "conv chain: layer too large");
        break;
      }
      ly.items = (int)items;
      if (ly.nkb > 1) {
        const DmaSplit sp = lat_split_plan(ly.d.M, ly.d.N, ly.d.K, 70 + rw);
        ly.d.ws = static_cast<float*>(alloc((size_t)sp.ws_floats * 4, false));
        ly.d.counters = static_cast<int*>(alloc((size_t)sp.counters * 4, true));
        if (!ly.d.ws || !ly.d.counters) {
          st = fail(RTENHIP_HIP_ERROR, "conv chain: hipMalloc failed");
          break;
        }
      }
      // Phase: one past the latest phase among the layers producing its
      // input and residual.
      for (int dv : {n.inputs[0], n.fused_residual}) {
        auto pr = producer.find(dv);
        if (dv >= 0 && pr != producer.end() && pr->second < L) phase[L] = std::max(phase[L], phase[pr->second] + 1);
      }
      in_r[L] = range_of(a.xin, a.N * a.C * a.Hp * a.Wp);
      res_r[L] = range_of(a.residual, a.N * a.O * g.oh * g.ow);
      out_r[L] = range_of(a.y, a.N * a.y_img);
    }
    // An arena-resident output must not overlap storage any other layer of
    // its phase or a later one reads or writes.
    bool ok = !st;
    for (int L = 0; ok && L < nl; L++) {
      if (!arena_out[L]) continue;
      for (int J = 0; ok && J < nl; J++)
        if (J != L && phase[J] >= phase[L] &&
            (in_r[J].overlaps(out_r[L]) || res_r[J].overlaps(out_r[L]) || out_r[J].overlaps(out_r[L])))
          ok = false;
    }
    if (!ok) {
      c.release();
      if (st) return st;
      continue;
    }
    // Tables: layers ordered by phase (run order inside a phase).
    std::vector<int> order(nl);
    for (int i = 0; i < nl; i++) order[i] = i;
    std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return phase[x] < phase[y]; });
    std::vector<ChainLayer> sorted;
    std::vector<ChainPhase> phases;
    for (int idx : order) {
      ChainLayer ly = layers[idx];
      while ((int)phases.size() <= phase[idx]) phases.push_back(ChainPhase{(int)sorted.size(), 0, 0});
      ChainPhase& ph = phases.back();
      ly.item_base = ph.items;
      ph.items += ly.items;
      ph.nl++;
      sorted.push_back(ly);
    }
    c.n_layers = nl;
    c.n_phases = (int)phases.size();
    RTENHIP_HIP_CHECK(hipMalloc(&c.layers_dev, sorted.size() * sizeof(ChainLayer)));
    RTENHIP_HIP_CHECK(hipMalloc(&c.phases_dev, phases.size() * sizeof(ChainPhase)));
    RTENHIP_HIP_CHECK(hipMalloc(&c.ctrl, (size_t)kChainCtrlInts * 4));
    RTENHIP_HIP_CHECK(hipMemsetAsync(c.ctrl, 0, (size_t)kChainCtrlInts * 4, s));
    RTENHIP_HIP_CHECK(hipMemcpyAsync(c.layers_dev, sorted.data(), sorted.size() * sizeof(ChainLayer),
                                     hipMemcpyHostToDevice, s));
    RTENHIP_HIP_CHECK(hipMemcpyAsync(c.phases_dev, phases.data(), phases.size() * sizeof(ChainPhase),
                                     hipMemcpyHostToDevice, s));
    RTENHIP_HIP_CHECK(hipStreamSynchronize(s));
    c.grid = conv_chain_grid();

    // One warm-up launch (surfaces a dependency timeout), then the chain
    // against its convs one by one (best of three each).
    rtenhip_status st2 = exec_chain(p, c);
    int err = 0;
    if (!st2 && (hipMemcpyAsync(&err, c.ctrl + chain_error_index(), 4, hipMemcpyDeviceToHost, s) != hipSuccess ||
                 hipStreamSynchronize(s) != hipSuccess))
      st2 = fail(RTENHIP_HIP_ERROR, "conv chain check failed");
    if (st2 || err) {
      c.release();
      if (st2) return st2;
      continue;
    }
    hipEvent_t e0 = nullptr, e1 = nullptr;
    RTENHIP_HIP_CHECK(hipEventCreate(&e0));
    RTENHIP_HIP_CHECK(hipEventCreate(&e1));
    auto time_it = [&](auto fn, float& best) -> rtenhip_status {
      best = 1e30f;
      for (int r = 0; r < 3; r++) {
        RTENHIP_HIP_CHECK(hipEventRecord(e0, s));
        rtenhip_status st3 = fn();
        if (st3) return st3;
        RTENHIP_HIP_CHECK(hipEventRecord(e1, s));
        RTENHIP_HIP_CHECK(hipEventSynchronize(e1));
        float t = 0;
        RTENHIP_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
        best = std::min(best, t);
      }
      return RTENHIP_OK;
    };
    st2 = time_it([&]() { return exec_chain(p, c); }, c.chain_ms);
    if (!st2)
      st2 = time_it(
          [&]() -> rtenhip_status {
            for (int op : c.ops) {
              rtenhip_status st4 = exec_op(p, op);
              if (st4) return st4;
            }
            return RTENHIP_OK;
          },
          c.ops_ms);
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (!st2 && hipMemcpyAsync(&err, c.ctrl + chain_error_index(), 4, hipMemcpyDeviceToHost, s) == hipSuccess &&
        hipStreamSynchronize(s) == hipSuccess && err)
      st2 = fail(RTENHIP_HIP_ERROR, "conv chain: a dependency wait timed out");
    if (getenv("RTENHIP_CHAIN_LOG"))
      fprintf(stderr, "conv chain: %d convs, %d phases, grid %d: chain %.4f ms vs convs one by one %.4f ms\n", nl,
              c.n_phases, c.grid, c.chain_ms, c.ops_ms);
    if (st2 || (chain_mode != 1 && c.chain_ms >= c.ops_ms)) {
      c.release();
      if (st2 && chain_mode == 1) return st2;
      continue;
    }
    const int idx = (int)p.chains.size();
    for (int op : c.ops) p.chain_of[op] = idx;
    p.chains.push_back(c);
  }
  return RTENHIP_OK;
}

rtenhip_status Graph::exec_chain(Plan& p, Plan::ConvChain& c) {
  (void)p;
  // Timing experiments: RTENHIP_CHAIN_STAMPS=<path> writes per-block phase
  // stamps {arrived, released} of eager launches to <path> (binary u64).
  static const char* stamp_path = getenv("RTENHIP_CHAIN_STAMPS");
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (stamp_path) (void)hipStreamIsCapturing(ctx->stream, &cs);
  const ChainLayer* ld = static_cast<const ChainLayer*>(c.layers_dev);
  const ChainPhase* pd = static_cast<const ChainPhase*>(c.phases_dev);
  if (!stamp_path || cs != hipStreamCaptureStatusNone)
    return launch_conv_chain(ld, pd, c.n_phases, c.ctrl, c.grid, ctx->stream);
  unsigned long long* st_dev = nullptr;
  const size_t bytes = (size_t)c.grid * c.n_phases * 48;  // barrier pairs, then 4 item stamps per block and phase
  RTENHIP_HIP_CHECK(hipMalloc(&st_dev, bytes));
  RTENHIP_HIP_CHECK(hipMemsetAsync(st_dev, 0, bytes, ctx->stream));
  rtenhip_status st = launch_conv_chain(ld, pd, c.n_phases, c.ctrl, c.grid, ctx->stream, st_dev);
  std::vector<unsigned long long> host(bytes / 8);
  if (!st && hipMemcpyAsync(host.data(), st_dev, bytes, hipMemcpyDeviceToHost, ctx->stream) == hipSuccess &&
      hipStreamSynchronize(ctx->stream) == hipSuccess) {
    if (FILE* f = fopen(stamp_path, "wb")) {
      const unsigned long long hdr[2] = {(unsigned long long)c.grid, (unsigned long long)c.n_phases};
      fwrite(hdr, 1, sizeof hdr, f);
      fwrite(host.data(), 1, bytes, f);
      fclose(f);
    }
  }
  (void)hipFree(st_dev);
  return st;
}

}  // namespace rtenhip
