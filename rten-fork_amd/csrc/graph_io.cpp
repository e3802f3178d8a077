// Host-resident and batch-sharded runs of the device graph on the C ABI.
//
// 1. rtenhip_graph_run_host / rtenhip_graph_wait: RTen's Model::run takes
//    host tensors and returns host tensors (src/model.rs:580-592), and
//    rten-cli times exactly that call (rten-cli/src/main.rs:296-317).  Done
//    naively (copy, run, copy, wait) every step pays its upload on top of the
//    forward: 38.5 MB per ResNet-50 batch of 64, ~0.7 ms of PCIe against a
//    ~5 ms forward.  HostPipe pipelines it inside the library: the inputs of
//    run k go from (pinned) host memory into device slot k % 2 on a
//    high-priority copy stream while run k - 1 computes, and run k's outputs
//    come back behind run k + 1's upload.  Events order the streams per slot,
//    so nothing waits on the host:
//
//      copy : wait in_free[s]   -> H2D inputs(k)  -> in_ready[s]
//             wait out_ready[s'] -> D2H outputs(k-1) -> out_free[s']
//      exec : wait in_ready[s], out_free[s] -> forward(slot s) -> in_free[s], out_ready[s]
//
//    The graph keeps one captured hipGraph per (input, output) binding
//    (Plan::captures), so the two slots replay without re-capturing.  The
//    copy stream is created at the highest priority: a process gets few
//    hardware queues (GPU_MAX_HW_QUEUES, 4 by default) and a normal-priority
//    stream can share the executor's queue, where the copies would wait behind
//    the forwards they are meant to overlap.
//
// 2. rtenhip_sharded_*: the graph runner sharding independent batch items over
//    the GPUs of one node (BASELINE.json north_star): one
//    replica of a .rten model per device, contiguous batch slices (earlier
//    shards take the remainder, like rten_hip/parallel.py shard_bounds), and
//    one exchange -- an RCCL all-gather of the per-shard outputs over xGMI when
//    the devices are distinct, else device-to-host copies of each shard into
//    the caller's output.  Batch items are independent (every conv / GEMM row
//    is per image, src/ops/conv.rs:243-270), so no collective runs on the data
//    path; each image's bits are those of the shard its device ran.
#include <dlfcn.h>

#include <cstdlib>

#include <algorithm>
#include <cstring>
#include <vector>

#include "graph.h"

namespace rtenhip {

struct HostPipe {
  static constexpr int kSlots = 2;
  int device = 0;
  hipStream_t copy = nullptr;
  struct Slot {
    std::vector<void*> in, out;  // device buffers
    hipEvent_t in_ready = nullptr, in_free = nullptr, out_ready = nullptr, out_free = nullptr;
  } slot[kSlots];
  std::vector<size_t> in_bytes, out_bytes;
  uint64_t k = 0;  // runs submitted
  // The download owed for the last submitted run (queued behind the next
  // upload, or by wait()).
  bool pending = false;
  int pending_slot = 0;
  std::vector<void*> pending_host;
  // Graph::run_seq of the run whose download is queued last, per slot.
  uint64_t slot_run[kSlots] = {0, 0};

  void free_buffers() {
    for (auto& s : slot) {
      for (void* p : s.in) (void)hipFree(p);
      for (void* p : s.out) (void)hipFree(p);
      s.in.clear();
      s.out.clear();
    }
    in_bytes.clear();
    out_bytes.clear();
  }
  ~HostPipe() {
    if (copy) (void)hipStreamSynchronize(copy);
    free_buffers();
    for (auto& s : slot)
      for (hipEvent_t e : {s.in_ready, s.in_free, s.out_ready, s.out_free})
        if (e) (void)hipEventDestroy(e);
    if (copy) (void)hipStreamDestroy(copy);
  }
};

void destroy_host_pipe(HostPipe* p) { delete p; }

static size_t tensor_bytes(const rtenhip_tensor& t) { return (size_t)numel(t) * 4; }

// Queue the owed download of the last run on the copy stream.
static rtenhip_status queue_download(HostPipe& hp) {
  if (!hp.pending) return RTENHIP_OK;
  HostPipe::Slot& s = hp.slot[hp.pending_slot];
  RTENHIP_HIP_CHECK(hipStreamWaitEvent(hp.copy, s.out_ready, 0));
  for (size_t j = 0; j < s.out.size(); j++)
    if (hp.out_bytes[j])
      RTENHIP_HIP_CHECK(hipMemcpyAsync(hp.pending_host[j], s.out[j], hp.out_bytes[j], hipMemcpyDeviceToHost, hp.copy));
  RTENHIP_HIP_CHECK(hipEventRecord(s.out_free, hp.copy));
  hp.pending = false;
  return RTENHIP_OK;
}

static rtenhip_status pipe_wait_all(Graph& g) {
  HostPipe* hp = g.host_pipe;
  rtenhip_status st = RTENHIP_OK;
  if (hp) {
    (void)hipSetDevice(hp->device);
    st = queue_download(*hp);
    if (hipStreamSynchronize(hp->copy) != hipSuccess && !st) st = fail(RTENHIP_HIP_ERROR, "hipStreamSynchronize");
  }
  const rtenhip_status s2 = g.synchronize();  // the executor, and deferred Gather checks
  return st ? st : s2;
}

static rtenhip_status run_host(Graph& g, const int32_t* in_ids, const rtenhip_tensor* ins, const int32_t* in_dt,
                               int n_in, const int32_t* out_ids, rtenhip_tensor* outs, int n_out, uint64_t* run_id) {
  if (n_in < 0 || n_out < 0 || (n_in && (!in_ids || !ins)) || (n_out && (!out_ids || !outs)))
    return fail(RTENHIP_INVALID_VALUE, "invalid run arguments");
  for (int i = 0; i < n_in; i++)
    if (!is_contiguous(ins[i]) || (numel(ins[i]) && !ins[i].data))
      return fail(RTENHIP_UNSUPPORTED_VALUE, "Host input must be a contiguous buffer");
  // Plan (shape-only; the host pointers are never dereferenced here).
  std::vector<int64_t> shapes((size_t)std::max(n_out, 1) * RTENHIP_MAX_DIMS);
  std::vector<int32_t> ndims((size_t)std::max(n_out, 1));
  rtenhip_status st = g.plan_shapes(in_ids, ins, n_in, out_ids, n_out, shapes.data(), ndims.data(), in_dt, nullptr);
  if (st) return st;
  std::vector<size_t> ib(n_in), ob(n_out);
  for (int i = 0; i < n_in; i++) ib[i] = tensor_bytes(ins[i]);
  for (int j = 0; j < n_out; j++) {
    if (outs[j].ndim != ndims[j] || !is_contiguous(outs[j]))
      return fail(RTENHIP_INCORRECT_OUTPUT_TYPE, "Output buffer has the wrong shape");
    for (int d = 0; d < ndims[j]; d++)
      if (outs[j].shape[d] != shapes[(size_t)j * RTENHIP_MAX_DIMS + d])
        return fail(RTENHIP_INCORRECT_OUTPUT_TYPE, "Output buffer has the wrong shape");
    ob[j] = tensor_bytes(outs[j]);
    if (ob[j] && !outs[j].data) return fail(RTENHIP_INVALID_VALUE, "Output buffer is NULL");
  }
  RTENHIP_HIP_CHECK(hipSetDevice(g.ctx->device));
  if (!g.host_pipe) {
    auto* hp = new HostPipe();
    hp->device = g.ctx->device;
    int lo = 0, hi = 0;
    (void)hipDeviceGetStreamPriorityRange(&lo, &hi);
    hipError_t e = hipStreamCreateWithPriority(&hp->copy, hipStreamNonBlocking, hi);
    for (auto& s : hp->slot)
      for (hipEvent_t* ev : {&s.in_ready, &s.in_free, &s.out_ready, &s.out_free})
        if (e == hipSuccess) e = hipEventCreateWithFlags(ev, hipEventDisableTiming);
    // Every event starts recorded (complete), so the first waits on them
    // are satisfied without relying on never-recorded-event semantics.
    for (auto& s : hp->slot)
      for (hipEvent_t ev : {s.in_ready, s.in_free, s.out_ready, s.out_free})
        if (e == hipSuccess) e = hipEventRecord(ev, hp->copy);
    if (e != hipSuccess) {
      delete hp;
      return hip_fail(e, "host pipeline setup");
    }
    g.host_pipe = hp;
  }
  HostPipe& hp = *g.host_pipe;
  if (hp.in_bytes != ib || hp.out_bytes != ob) {
    // New shapes: settle every queued run, then re-size the slot buffers.
    if ((st = pipe_wait_all(g))) return st;
    hp.free_buffers();
    for (auto& s : hp.slot) {
      for (size_t b : ib) {
        void* p = nullptr;
        RTENHIP_HIP_CHECK(hipMalloc(&p, std::max<size_t>(b, 4)));
        s.in.push_back(p);
      }
      for (size_t b : ob) {
        void* p = nullptr;
        RTENHIP_HIP_CHECK(hipMalloc(&p, std::max<size_t>(b, 4)));
        s.out.push_back(p);
      }
    }
    hp.in_bytes = ib;
    hp.out_bytes = ob;
  }
  const int si = (int)(hp.k % HostPipe::kSlots);
  HostPipe::Slot& s = hp.slot[si];
  // Upload into the slot once the forward that last read it is done.
  RTENHIP_HIP_CHECK(hipStreamWaitEvent(hp.copy, s.in_free, 0));
  for (int i = 0; i < n_in; i++)
    if (ib[i]) RTENHIP_HIP_CHECK(hipMemcpyAsync(s.in[i], ins[i].data, ib[i], hipMemcpyHostToDevice, hp.copy));
  RTENHIP_HIP_CHECK(hipEventRecord(s.in_ready, hp.copy));
  // The previous run's outputs go back behind this upload.
  if ((st = queue_download(hp))) return st;
  std::vector<rtenhip_tensor> din(n_in), dout(n_out);
  for (int i = 0; i < n_in; i++) {
    din[i] = ins[i];
    din[i].data = static_cast<float*>(s.in[i]);
  }
  for (int j = 0; j < n_out; j++) {
    dout[j] = outs[j];
    dout[j].data = static_cast<float*>(s.out[j]);
  }
  g.ext_order = true;
  g.ext_waits = {s.in_ready, s.out_free};
  g.ext_records = {s.in_free, s.out_ready};
  // The run must not wait on the host for its Gather check: the check is
  // queued and reported by rtenhip_graph_wait (as in deferred mode).
  const bool deferred = g.deferred_checks;
  g.deferred_checks = true;
  st = g.run(in_ids, din.data(), n_in, out_ids, dout.data(), n_out, in_dt);
  g.deferred_checks = deferred;
  g.ext_order = false;
  g.ext_waits.clear();
  g.ext_records.clear();
  if (st) return st;
  hp.pending = true;
  hp.pending_slot = si;
  hp.pending_host.assign(n_out, nullptr);
  for (int j = 0; j < n_out; j++) hp.pending_host[j] = outs[j].data;
  hp.slot_run[si] = g.run_seq;
  hp.k++;
  if (run_id) *run_id = g.run_seq;
  return RTENHIP_OK;
}

static rtenhip_status wait_run(Graph& g, uint64_t run) {
  HostPipe* hp = g.host_pipe;
  if (run == 0 || !hp) return pipe_wait_all(g);
  if (run > g.run_seq) return fail(RTENHIP_INVALID_VALUE, "unknown run id");
  RTENHIP_HIP_CHECK(hipSetDevice(hp->device));
  rtenhip_status st = RTENHIP_OK;
  const int si = (int)((hp->k + HostPipe::kSlots - 1) % HostPipe::kSlots);  // the last submitted run's slot
  if (hp->pending && run >= hp->slot_run[si]) st = queue_download(*hp);
  if (st) return st;
  // out_free of a slot is recorded (in copy-stream order) after the download
  // of the newest run that used it, so it covers every older run too.
  for (auto& s : hp->slot) RTENHIP_HIP_CHECK(hipEventSynchronize(s.out_free));
  // Gather checks of finished runs (their events precede out_ready).
  for (auto& pl : g.plans)
    if (pl->gather_flag) {
      const rtenhip_status s2 = g.collect_gather_checks(*pl, false);
      if (s2) return s2;
    }
  if (g.deferred_error_run && g.deferred_error_run <= run) {
    g.deferred_error_run = 0;
    return fail(RTENHIP_INVALID_VALUE, "Entry in `indices` is out of range");
  }
  return RTENHIP_OK;
}

// ---- batch-sharded runner ---------------------------------------------------

// RCCL, loaded at run time: the copy already in the process when there is
// one (torch's, same soname), else the system library.  The library does not
// link it, so the single-GPU paths never depend on it.
struct Rccl {
  void* lib = nullptr;
  typedef int (*InitAll)(void** comms, int ndev, const int* devs);
  typedef int (*AllGather)(const void* send, void* recv, size_t count, int dtype, void* comm, hipStream_t s);
  typedef int (*Group)();
  typedef int (*Destroy)(void* comm);
  typedef const char* (*ErrStr)(int);
  InitAll init_all = nullptr;
  AllGather all_gather = nullptr;
  Group group_start = nullptr, group_end = nullptr;
  Destroy destroy = nullptr;
  ErrStr err = nullptr;
  bool load() {
    if (lib) return true;
    for (const char* name : {"librccl.so.1", "/opt/rocm/lib/librccl.so.1", "librccl.so"}) {
      lib = dlopen(name, RTLD_NOW | RTLD_NOLOAD);
      if (!lib) lib = dlopen(name, RTLD_NOW | RTLD_LOCAL);
      if (lib) break;
    }
    if (!lib) return false;
    init_all = reinterpret_cast<InitAll>(dlsym(lib, "ncclCommInitAll"));
    all_gather = reinterpret_cast<AllGather>(dlsym(lib, "ncclAllGather"));
    group_start = reinterpret_cast<Group>(dlsym(lib, "ncclGroupStart"));
    group_end = reinterpret_cast<Group>(dlsym(lib, "ncclGroupEnd"));
    destroy = reinterpret_cast<Destroy>(dlsym(lib, "ncclCommDestroy"));
    err = reinterpret_cast<ErrStr>(dlsym(lib, "ncclGetErrorString"));
    return init_all && all_gather && group_start && group_end && destroy;
  }
};
constexpr int kNcclFloat32 = 7;  // ncclDataType_t ncclFloat32 (rccl.h)

struct Sharded {
  std::vector<int> devices;
  std::vector<rtenhip_ctx*> ctxs;
  std::vector<rtenhip_graph*> graphs;
  std::vector<hipStream_t> streams;
  bool rccl = false;
  Rccl nccl;
  std::vector<void*> comms;
  // Per shard: device input / output (rows = the largest shard, so the
  // all-gather sends equal counts), and the gathered outputs [n][rows][...].
  std::vector<void*> din, dout, gathered;
  int64_t rows = -1, in_row = -1, out_row = -1;
  std::vector<int64_t> out_inner;  // output shape after the batch dim

  void free_buffers() {
    for (size_t i = 0; i < devices.size(); i++) {
      (void)hipSetDevice(devices[i]);
      for (auto* v : {&din, &dout, &gathered})
        if (i < v->size() && (*v)[i]) (void)hipFree((*v)[i]);
    }
    din.clear();
    dout.clear();
    gathered.clear();
    rows = -1;
  }
  ~Sharded() {
    for (size_t i = 0; i < devices.size(); i++) {
      (void)hipSetDevice(devices[i]);
      if (i < streams.size() && streams[i]) (void)hipStreamSynchronize(streams[i]);
    }
    free_buffers();
    for (void* c : comms)
      if (c && nccl.destroy) nccl.destroy(c);
    for (size_t i = 0; i < devices.size(); i++) {
      (void)hipSetDevice(devices[i]);
      if (i < graphs.size() && graphs[i]) rtenhip_graph_destroy(graphs[i]);
      if (i < ctxs.size() && ctxs[i]) rtenhip_destroy(ctxs[i]);
      if (i < streams.size() && streams[i]) (void)hipStreamDestroy(streams[i]);
    }
  }
};

// [start, end) of shard r of `total` items over `world` shards
// (rten_hip/parallel.py shard_bounds).
static void shard_bounds(int64_t total, int r, int world, int64_t& a, int64_t& b) {
  const int64_t base = total / world, rem = total % world;
  a = r * base + std::min<int64_t>(r, rem);
  b = a + base + (r < rem ? 1 : 0);
}

static rtenhip_status sharded_run_host(Sharded& sh, const rtenhip_tensor* x, rtenhip_tensor* y) {
  const int n = (int)sh.devices.size();
  if (!x || !y || x->ndim < 1 || !is_contiguous(*x) || !is_contiguous(*y) || (numel(*x) && !x->data))
    return fail(RTENHIP_INVALID_VALUE, "invalid sharded run arguments");
  const int64_t total = x->shape[0];
  int64_t in_row = 1;
  for (int d = 1; d < x->ndim; d++) in_row *= x->shape[d];
  const int64_t rows = (total + n - 1) / n;
  Graph& g0 = *reinterpret_cast<Graph*>(sh.graphs[0]);
  const int32_t in_id = g0.model_inputs.at(0), out_id = g0.model_outputs.at(0);
  // Output shape per image: plan the largest shard on shard 0.
  rtenhip_tensor xs = *x;
  xs.shape[0] = std::max<int64_t>(rows, 1);
  int64_t oshape[RTENHIP_MAX_DIMS];
  int32_t ondim = 0;
  rtenhip_status st = g0.plan_shapes(&in_id, &xs, 1, &out_id, 1, oshape, &ondim);
  if (st) return st;
  if (ondim < 1 || oshape[0] != xs.shape[0]) return fail(RTENHIP_UNSUPPORTED_VALUE, "model output is not batched");
  int64_t out_row = 1;
  for (int d = 1; d < ondim; d++) out_row *= oshape[d];
  if (y->ndim != ondim || y->shape[0] != total) return fail(RTENHIP_INCORRECT_OUTPUT_TYPE, "Output buffer has the wrong shape");
  for (int d = 1; d < ondim; d++)
    if (y->shape[d] != oshape[d]) return fail(RTENHIP_INCORRECT_OUTPUT_TYPE, "Output buffer has the wrong shape");
  if (numel(*y) && !y->data) return fail(RTENHIP_INVALID_VALUE, "Output buffer is NULL");
  if (total == 0) return RTENHIP_OK;
  if (rows != sh.rows || in_row != sh.in_row || out_row != sh.out_row) {
    sh.free_buffers();
    sh.din.assign(n, nullptr);
    sh.dout.assign(n, nullptr);
    sh.gathered.assign(n, nullptr);
    for (int i = 0; i < n; i++) {
      RTENHIP_HIP_CHECK(hipSetDevice(sh.devices[i]));
      RTENHIP_HIP_CHECK(hipMalloc(&sh.din[i], std::max<size_t>((size_t)(rows * in_row) * 4, 4)));
      RTENHIP_HIP_CHECK(hipMalloc(&sh.dout[i], std::max<size_t>((size_t)(rows * out_row) * 4, 4)));
      // (padding rows of a short shard: zeros, so the gathered buffer is defined)
      RTENHIP_HIP_CHECK(hipMemsetAsync(sh.dout[i], 0, (size_t)(rows * out_row) * 4, sh.streams[i]));
      if (sh.rccl) RTENHIP_HIP_CHECK(hipMalloc(&sh.gathered[i], (size_t)(n * rows * out_row) * 4));
    }
    sh.rows = rows;
    sh.in_row = in_row;
    sh.out_row = out_row;
  }
  // Upload each shard and queue its forward (asynchronous after a plan's
  // first, tuning run).
  for (int i = 0; i < n; i++) {
    int64_t a, b;
    shard_bounds(total, i, n, a, b);
    if (b == a) continue;
    RTENHIP_HIP_CHECK(hipSetDevice(sh.devices[i]));
    const float* src = x->data + a * in_row;
    RTENHIP_HIP_CHECK(hipMemcpyAsync(sh.din[i], src, (size_t)((b - a) * in_row) * 4, hipMemcpyHostToDevice, sh.streams[i]));
    rtenhip_tensor xi = *x;
    xi.data = static_cast<float*>(sh.din[i]);
    xi.shape[0] = b - a;
    xi.strides[0] = in_row;
    rtenhip_tensor yi = make_tensor(static_cast<float*>(sh.dout[i]), oshape, ondim);
    yi.shape[0] = b - a;
    st = rtenhip_graph_run(sh.graphs[i], &in_id, &xi, 1, &out_id, &yi, 1);
    if (st) return st;
  }
  if (sh.rccl) {
    // The one exchange: all-gather of every shard's (padded) output rows.
    if (sh.nccl.group_start() != 0) return fail(RTENHIP_HIP_ERROR, "ncclGroupStart failed");
    int rc = 0;
    for (int i = 0; i < n && !rc; i++) {
      (void)hipSetDevice(sh.devices[i]);
      rc = sh.nccl.all_gather(sh.dout[i], sh.gathered[i], (size_t)(rows * out_row), kNcclFloat32, sh.comms[i],
                              sh.streams[i]);
    }
    const int rc2 = sh.nccl.group_end();
    if (rc || rc2) {
      set_error(RTENHIP_HIP_ERROR, std::string("ncclAllGather failed: ") +
                                       (sh.nccl.err ? sh.nccl.err(rc ? rc : rc2) : "unknown error"));
      return RTENHIP_HIP_ERROR;
    }
    RTENHIP_HIP_CHECK(hipSetDevice(sh.devices[0]));
    for (int r = 0; r < n; r++) {
      int64_t a, b;
      shard_bounds(total, r, n, a, b);
      if (b > a)
        RTENHIP_HIP_CHECK(hipMemcpyAsync(y->data + a * out_row, static_cast<float*>(sh.gathered[0]) + r * rows * out_row,
                                         (size_t)((b - a) * out_row) * 4, hipMemcpyDeviceToHost, sh.streams[0]));
    }
  } else {
    for (int i = 0; i < n; i++) {
      int64_t a, b;
      shard_bounds(total, i, n, a, b);
      if (b == a) continue;
      RTENHIP_HIP_CHECK(hipSetDevice(sh.devices[i]));
      RTENHIP_HIP_CHECK(hipMemcpyAsync(y->data + a * out_row, sh.dout[i], (size_t)((b - a) * out_row) * 4,
                                       hipMemcpyDeviceToHost, sh.streams[i]));
    }
  }
  // Model::run returns when the outputs are on the host.
  for (int i = 0; i < n; i++) {
    RTENHIP_HIP_CHECK(hipSetDevice(sh.devices[i]));
    RTENHIP_HIP_CHECK(hipStreamSynchronize(sh.streams[i]));
    st = rtenhip_graph_synchronize(sh.graphs[i]);
    if (st) return st;
  }
  return RTENHIP_OK;
}

}  // namespace rtenhip

using namespace rtenhip;

extern "C" {

void* rtenhip_host_alloc(rtenhip_ctx* ctx, size_t bytes) {
  if (ctx && hipSetDevice(reinterpret_cast<Ctx*>(ctx)->device) != hipSuccess) return nullptr;
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 4, hipHostMallocDefault) != hipSuccess) {
    set_error(RTENHIP_HIP_ERROR, "hipHostMalloc failed");
    return nullptr;
  }
  return p;
}

void rtenhip_host_free(rtenhip_ctx*, void* ptr) {
  if (ptr) (void)hipHostFree(ptr);
}

rtenhip_status rtenhip_graph_run_host(rtenhip_graph* g, const int32_t* input_ids, const rtenhip_tensor* inputs,
                                      const int32_t* input_dtypes, int32_t n_inputs, const int32_t* output_ids,
                                      rtenhip_tensor* outputs, int32_t n_outputs, uint64_t* run_id) {
  if (!g) return fail(RTENHIP_INVALID_VALUE, "graph is NULL");
  return run_host(*reinterpret_cast<Graph*>(g), input_ids, inputs, input_dtypes, n_inputs, output_ids, outputs,
                  n_outputs, run_id);
}

rtenhip_status rtenhip_graph_wait(rtenhip_graph* g, uint64_t run_id) {
  if (!g) return fail(RTENHIP_INVALID_VALUE, "graph is NULL");
  return wait_run(*reinterpret_cast<Graph*>(g), run_id);
}

rtenhip_sharded* rtenhip_sharded_create(const uint8_t* bytes, size_t len, const int32_t* devices, int32_t n_devices,
                                        int optimize) {
  if (!bytes || !devices || n_devices < 1) {
    set_error(RTENHIP_INVALID_VALUE, "invalid sharded runner arguments");
    return nullptr;
  }
  auto* sh = new Sharded();
  for (int i = 0; i < n_devices; i++) {
    sh->devices.push_back(devices[i]);
    rtenhip_ctx* c = rtenhip_create(devices[i]);
    sh->ctxs.push_back(c);
    hipStream_t s = nullptr;
    if (!c || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
      if (c) set_error(RTENHIP_HIP_ERROR, "hipStreamCreate failed");
      delete sh;
      return nullptr;
    }
    sh->streams.push_back(s);
    (void)rtenhip_set_stream(c, s);
    rtenhip_graph* g = rtenhip_model_load_with_options(c, bytes, len, optimize);
    sh->graphs.push_back(g);
    if (!g) {
      delete sh;
      return nullptr;
    }
    const Graph& gg = *reinterpret_cast<Graph*>(g);
    if (gg.model_inputs.size() != 1 || gg.model_outputs.size() != 1) {
      set_error(RTENHIP_UNSUPPORTED_VALUE, "sharded runs take models with one input and one output");
      delete sh;
      return nullptr;
    }
  }
  std::vector<int> d = sh->devices;
  std::sort(d.begin(), d.end());
  const bool distinct = std::adjacent_find(d.begin(), d.end()) == d.end();
  const char* env = getenv("RTENHIP_SHARDED_RCCL");
  if (n_devices > 1 && distinct && !(env && env[0] == '0')) {
    if (!sh->nccl.load()) {
      set_error(RTENHIP_HIP_ERROR, "RCCL (librccl.so.1) not found for the all-gather over distinct devices");
      delete sh;
      return nullptr;
    }
    sh->comms.assign(n_devices, nullptr);
    const int rc = sh->nccl.init_all(sh->comms.data(), n_devices, sh->devices.data());
    if (rc != 0) {
      set_error(RTENHIP_HIP_ERROR, std::string("ncclCommInitAll failed: ") + (sh->nccl.err ? sh->nccl.err(rc) : "?"));
      sh->comms.clear();
      delete sh;
      return nullptr;
    }
    sh->rccl = true;
  }
  return reinterpret_cast<rtenhip_sharded*>(sh);
}

void rtenhip_sharded_destroy(rtenhip_sharded* s) { delete reinterpret_cast<Sharded*>(s); }

int32_t rtenhip_sharded_gather_mode(rtenhip_sharded* s) { return s && reinterpret_cast<Sharded*>(s)->rccl ? 1 : 0; }

rtenhip_graph* rtenhip_sharded_graph(rtenhip_sharded* s, int32_t shard) {
  Sharded* sh = reinterpret_cast<Sharded*>(s);
  if (!sh || shard < 0 || shard >= (int)sh->graphs.size()) return nullptr;
  return sh->graphs[shard];
}

rtenhip_status rtenhip_sharded_run_host(rtenhip_sharded* s, const rtenhip_tensor* input, rtenhip_tensor* output) {
  if (!s) return fail(RTENHIP_INVALID_VALUE, "sharded runner is NULL");
  return sharded_run_host(*reinterpret_cast<Sharded*>(s), input, output);
}

const float* rtenhip_sharded_gathered(rtenhip_sharded* s, int32_t shard) {
  Sharded* sh = reinterpret_cast<Sharded*>(s);
  if (!sh || !sh->rccl || shard < 0 || shard >= (int)sh->gathered.size()) return nullptr;
  return static_cast<const float*>(sh->gathered[shard]);
}

}  // extern "C"
