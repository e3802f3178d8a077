// Conv chains of a plan (ConvChain, conv_chain.hip): which runs of convs
// become one persistent launch, their layer descriptors and dependencies,
// and the build-time check that the chain beats the convs one by one.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
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
// that (a) the plan runs on the DMA or latency GEMM (tuned on the first run),
// ungrouped, not an FC layer, not part of an expand+depthwise fusion or a
// broadcast residual; (b) read an input that needs no padding copy (unpadded
// or zero-bordered by its producer); (c) touch no graph input or output (the
// descriptors hold plan-fixed pointers).  A run becomes a chain when at least
// half of its convs were tuned to the latency GEMM (small batches) or
// RTENHIP_CHAIN=1; it is kept when one launch of it times faster than its
// convs one by one (RTENHIP_CHAIN=1 keeps it regardless).  Values the chain
// both produces and consumes get chain-owned storage, so only the outputs
// that leave the chain can overwrite storage an earlier layer used (those
// become whole-layer dependencies); the rest are per-region (ChainLayer).
rtenhip_status Graph::build_chains(Plan& p) {
  for (auto& c : p.chains) c.release();
  p.chains.clear();
  p.chain_of.clear();
  p.chains_built = true;
  p.chains_arena = arena;
  if (chain_mode == 0) return RTENHIP_OK;
  std::set<int> io(p.input_ids.begin(), p.input_ids.end());
  io.insert(p.output_ids.begin(), p.output_ids.end());
  auto eligible = [&](int op) {
    auto it = p.convs.find(op);
    if (it == p.convs.end()) return false;
    const ConvExec& ce = it->second;
    if (ce.fc || ce.cfg < 0 || ce.cfg >= kPwCfgBase || ce.g.groups != 1) return false;
    if (p.expand_fused.count(op) || p.conv_unfused.count(op)) return false;
    if (p.dual_on.count(op) || p.dual_skip.count(op)) return false;
    const Node& n = nodes[op];
    const ConvPlan& g = ce.g;
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

  hipStream_t s = ctx->stream;
  // Consumers of each value among the plan's ops.
  std::map<int, std::vector<int>> consumers;
  for (int op : p.ops) {
    const Node& n = nodes[op];
    for (int v : n.inputs)
      if (v >= 0) consumers[v].push_back(op);
    if (n.fused_residual >= 0) consumers[n.fused_residual].push_back(op);
  }
  for (const std::vector<int>& run : runs) {
    int lat = 0;
    for (int op : run) lat += is_lat_cfg(p.convs[op].cfg) ? 1 : 0;
    if (chain_mode != 1 && 2 * lat < (int)run.size()) continue;
    ConvChain c;
    c.ops = run;
    const std::set<int> in_run(run.begin(), run.end());
    std::map<int, int> producer;  // value -> layer index
    for (size_t i = 0; i < run.size(); i++) producer[nodes[run[i]].outputs[0]] = (int)i;
    // Values produced and consumed only inside the chain get storage of their
    // own (no reuse, so no write-after-read ordering inside the launch).
    std::map<int, float*> priv;
    rtenhip_status st = RTENHIP_OK;
    for (int op : run) {
      const int v = nodes[op].outputs[0];
      if (p.padded.count(v)) continue;
      bool inside = consumers.count(v) > 0;
      for (int cop : consumers[v]) inside = inside && in_run.count(cop) > 0;
      if (!inside) continue;
      const ConvPlan& g = p.convs[op].g;
      float* b = nullptr;
      if (hipMalloc(&b, (size_t)(g.N * g.O * g.oh * g.ow) * 4) != hipSuccess) {
        st = fail(RTENHIP_HIP_ERROR, "conv chain: hipMalloc failed");
        break;
      }
      c.packed.push_back(b);  // chain-owned device buffers
      priv[v] = b;
    }
    std::vector<ChainLayer> layers;
    std::vector<Range> in_r, res_r, out_r;
    int64_t ws_floats = 0, n_counters = 0, n_tilecnt = 0;
    std::vector<int64_t> ws_off, cnt_off;
    bool ok = !st;
    for (size_t L = 0; ok && L < run.size(); L++) {
      const int op = run[L];
      const Node& n = nodes[op];
      ConvExec& ce = p.convs[op];
      const ConvPlan& g = ce.g;
      ConvDmaArgs a{};
      conv_io_args(p, op, a);
      if (priv.count(n.inputs[0])) a.xin = priv[n.inputs[0]];
      if (n.fused_residual >= 0 && priv.count(n.fused_residual)) a.residual = priv[n.fused_residual];
      if (priv.count(n.outputs[0])) {
        a.y = priv[n.outputs[0]];
        a.y_img = g.O * g.oh * g.ow;
        a.y_row = a.y_off = 0;
      }
      if (is_lat_cfg(ce.cfg)) {
        a.packed_w = ce.packed;
      } else {
        float* pk = nullptr;
        RTENHIP_HIP_CHECK(hipMalloc(&pk, (size_t)packed_conv_weight_floats(g, kLatCfgBase + 41) * 4));
        c.packed.push_back(pk);
        if ((st = pack_conv_weights(ctx, ptr_of(p, n.inputs[1]), g, kLatCfgBase + 41, pk))) return st;
        a.packed_w = pk;
      }
      ChainLayer ly{};
      if ((st = lat_conv_desc(ctx, a, ly.d))) return st;
      ly.subs = (ly.d.M + 15) / 16;
      ly.n16 = (ly.d.N + 15) / 16;
      ly.nkb = (ly.d.K + 255) / 256;
      ly.tiles = ly.subs * ly.n16;
      ly.items = ly.tiles * ly.nkb;
      ly.item_base = c.items;
      const int64_t P = g.oh * g.ow;
      ly.dep_x = producer.count(n.inputs[0]) && producer[n.inputs[0]] < (int)L ? producer[n.inputs[0]] : -1;
      ly.dep_r = n.fused_residual >= 0 && producer.count(n.fused_residual) && producer[n.fused_residual] < (int)L
                     ? producer[n.fused_residual]
                     : -1;
      ly.in_H = (int)g.H;
      ly.in_W = (int)g.W;
      ly.in_P = (int)(g.H * g.W);
      ly.S = (int)g.sh;
      ly.pt = (int)g.pads[0];
      ly.kext = (int)((g.kh - 1) * g.dh + 1);
      ly.OW = (int)g.ow;
      ly.P = (int)P;
      const Range xin = range_of(a.xin, a.N * a.C * a.Hp * a.Wp);
      const Range res = range_of(a.residual, a.N * a.O * P);
      const Range out = range_of(a.y, a.N * a.y_img);
      // Layer dependencies: earlier layers that read or write the storage this
      // conv overwrites (never the case for chain-private outputs).
      std::vector<int> deps;
      for (size_t j = 0; j < layers.size(); j++)
        if (in_r[j].overlaps(out) || res_r[j].overlaps(out) || out_r[j].overlaps(out)) deps.push_back((int)j);
      if ((int)deps.size() > kChainMaxDeps || (int64_t)c.items + ly.items > 0x7fffffff) {
        ok = false;
        break;
      }
      ly.ndeps = (int)deps.size();
      for (size_t k = 0; k < deps.size(); k++) {
        ly.deps[k] = deps[k];
        layers[deps[k]].layer_word = 1;
      }
      c.items += ly.items;
      ws_off.push_back(ws_floats);
      if (ly.nkb > 1) {
        ws_floats += (int64_t)ly.tiles * ly.nkb * 256;
        n_counters += ly.tiles;
      }
      cnt_off.push_back(n_tilecnt);
      n_tilecnt += (int64_t)ly.n16 * kChainTileStride;
      layers.push_back(ly);
      in_r.push_back(xin);
      res_r.push_back(res);
      out_r.push_back(out);
    }
    if (!ok || st) {
      c.release();
      if (st) return st;
      continue;
    }
    const int nl = (int)layers.size();
    const int64_t base = chain_counters_base(nl);
    c.ctrl_bytes = (size_t)(base + n_counters + n_tilecnt) * 4;
    RTENHIP_HIP_CHECK(hipMalloc(&c.layers_dev, (size_t)nl * sizeof(ChainLayer)));
    RTENHIP_HIP_CHECK(hipMalloc(&c.ctrl, c.ctrl_bytes));
    if (ws_floats) RTENHIP_HIP_CHECK(hipMalloc(&c.ws, (size_t)ws_floats * 4));
    int64_t split_off = 0;
    for (int i = 0; i < nl; i++) {
      if (layers[i].nkb > 1) {
        layers[i].d.ws = c.ws + ws_off[i];
        layers[i].d.counters = c.ctrl + base + split_off;
        split_off += layers[i].tiles;
      }
      layers[i].cnt_base = (int)(base + n_counters + cnt_off[i]);
    }
    RTENHIP_HIP_CHECK(hipMemcpy(c.layers_dev, layers.data(), (size_t)nl * sizeof(ChainLayer), hipMemcpyHostToDevice));
    c.grid = conv_chain_grid();
    const int idx = (int)p.chains.size();
    for (int op : c.ops) p.chain_of[op] = idx;
    p.chains.push_back(c);
  }
  if (p.chains.empty()) return RTENHIP_OK;

  // Chain members run on the main stream, in the chain.
  for (auto& kv : p.chain_of) {
    p.side.erase(kv.first);
    for (auto& j : p.joins) j.second.erase(std::remove(j.second.begin(), j.second.end(), kv.first), j.second.end());
  }

  // One warm-up launch (surfaces a dependency timeout), then the timing
  // comparison: the chain vs its convs launched one by one.
  hipEvent_t e0 = nullptr, e1 = nullptr;
  RTENHIP_HIP_CHECK(hipEventCreate(&e0));
  RTENHIP_HIP_CHECK(hipEventCreate(&e1));
  rtenhip_status st = RTENHIP_OK;
  for (ConvChain& c : p.chains) {
    c.use = true;
    if ((st = exec_chain(p, c))) break;
    int err = 0;
    if (hipMemcpyAsync(&err, c.ctrl + chain_error_index((int)c.ops.size()), 4, hipMemcpyDeviceToHost, s) !=
            hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) {
      st = fail(RTENHIP_HIP_ERROR, "conv chain check failed");
      break;
    }
    if (err) {
      c.release();
      continue;
    }
    auto time_it = [&](auto fn, float& best) -> rtenhip_status {
      best = 1e30f;
      for (int r = 0; r < 3; r++) {
        RTENHIP_HIP_CHECK(hipEventRecord(e0, s));
        rtenhip_status st2 = fn();
        if (st2) return st2;
        RTENHIP_HIP_CHECK(hipEventRecord(e1, s));
        RTENHIP_HIP_CHECK(hipEventSynchronize(e1));
        float t = 0;
        RTENHIP_HIP_CHECK(hipEventElapsedTime(&t, e0, e1));
        best = std::min(best, t);
      }
      return RTENHIP_OK;
    };
    if ((st = time_it([&]() { return exec_chain(p, c); }, c.chain_ms))) break;
    if ((st = time_it(
             [&]() -> rtenhip_status {
               for (int op : c.ops) {
                 rtenhip_status st3 = exec_op(p, op);
                 if (st3) return st3;
               }
               return RTENHIP_OK;
             },
             c.ops_ms)))
      break;
    if (chain_mode != 1 && c.chain_ms >= c.ops_ms) c.release();
  }
  (void)hipEventDestroy(e0);
  (void)hipEventDestroy(e1);
  return st;
}

rtenhip_status Graph::exec_chain(Plan& p, ConvChain& c) {
  RTENHIP_HIP_CHECK(hipMemsetAsync(c.ctrl, 0, c.ctrl_bytes, ctx->stream));
  // Timing experiments: RTENHIP_CHAIN_STAMPS=<path> writes per-unit
  // timestamps of eager launches to <path>.<chain index> (binary u64 x 4).
  static const char* stamp_path = getenv("RTENHIP_CHAIN_STAMPS");
  hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
  if (stamp_path) (void)hipStreamIsCapturing(ctx->stream, &cs);
  if (!stamp_path || cs != hipStreamCaptureStatusNone)
    return launch_conv_chain(static_cast<const ChainLayer*>(c.layers_dev), (int)c.ops.size(), c.items, c.ctrl,
                             c.grid, ctx->stream);
  unsigned long long* st_dev = nullptr;
  const size_t bytes = (size_t)c.items * 32;
  RTENHIP_HIP_CHECK(hipMalloc(&st_dev, bytes));
  rtenhip_status st = launch_conv_chain(static_cast<const ChainLayer*>(c.layers_dev), (int)c.ops.size(), c.items,
                                        c.ctrl, c.grid, ctx->stream, st_dev);
  std::vector<unsigned long long> host(bytes / 8);
  if (!st && hipMemcpyAsync(host.data(), st_dev, bytes, hipMemcpyDeviceToHost, ctx->stream) == hipSuccess &&
      hipStreamSynchronize(ctx->stream) == hipSuccess) {
    int idx = 0;
    for (size_t i = 0; i < p.chains.size(); i++)
      if (&p.chains[i] == &c) idx = (int)i;
    const std::string path = std::string(stamp_path) + "." + std::to_string(idx);
    if (FILE* f = fopen(path.c_str(), "wb")) {
      fwrite(host.data(), 1, bytes, f);
      fclose(f);
    }
  }
  (void)hipFree(st_dev);
  return st;
}

}  // namespace rtenhip
