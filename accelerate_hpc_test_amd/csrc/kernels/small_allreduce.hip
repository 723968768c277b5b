// One-shot all-reduce for small messages (<= 1 MiB) between the GPUs of one node, over buffers the ranks map into each
// other's address space with HIP IPC (xGMI peer loads / stores), not through an RCCL ring. For the latency-bound
// collectives of a training step — the clip-norm scalar, loss / metric reductions, `check_trigger` flags, fp8 amax
// vectors — one kernel does the whole collective: every rank pushes its input into its OWN buffer, raises one flag per
// workgroup in every peer's buffer, waits for the peers' flags in its own (local polling), then reads the peers'
// copies and reduces them in registers. No ring steps, no proxy thread, one launch.
//
// Memory: each rank's buffer is allocated uncached (hipDeviceMallocUncached), so flag polls and peer data reads see
// the other GPUs' stores without cache maintenance; the writer orders "data, then flag" with a system-scope release.
// Buffer layout: flags [kMaxRanks][kMaxBlocks] (uint32, value = call epoch) | data slot 0 | data slot 1. Consecutive
// calls alternate data slots: a rank can start call e+1 while a slow peer still reads call e's slot, and it cannot
// reach call e+2 (same slot as e) before every peer raised its e+1 flags, i.e. finished reading e.
//
// Every wait is bounded (a few seconds of polling); on timeout the kernel records an error in a host-mapped word and
// returns, so a missing peer never leaves a workgroup spinning past the process (the host raises on the next check).
#include <hip/hip_runtime.h>
#include <torch/extension.h>
#include <ATen/hip/HIPContext.h>
#include "common.h"
#include <limits>
#include <map>
#include <type_traits>
#include <mutex>
#include <string>
#include <vector>

using namespace acc;

namespace {

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 64;
constexpr int kFlagBytes = kMaxRanks * kMaxBlocks * 4;
constexpr int kThreads = 512;

struct Peers {
  uint8_t* buf[kMaxRanks];
};

enum Op { kSum = 0, kMax = 1 };

template <typename T> struct Acc { using type = float; };
template <> struct Acc<int64_t> { using type = int64_t; };
template <> struct Acc<int32_t> { using type = int64_t; };

template <typename T> __device__ __forceinline__ typename Acc<T>::type load_acc(const T* p) { return (typename Acc<T>::type)(*p); }
template <> __device__ __forceinline__ float load_acc<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T> __device__ __forceinline__ T store_cast(typename Acc<T>::type v) { return (T)v; }
template <> __device__ __forceinline__ bf16_t store_cast<bf16_t>(float v) { return f2bf(v); }

// Per-launch inputs / outputs: entry y serves rank rank0 + y (gridDim.y = 1 in a real rank; the single-process
// virtual-peer test runs every rank's workgroups in ONE launch so they are co-resident).
struct IO {
  const void* in[kMaxRanks];
  void* out[kMaxRanks];
};

template <typename T>
__device__ inline T poison() {
  // bf16_t is raw uint16 storage: it is a float type here (the Acc<T> of every float type is float)
  if constexpr (std::is_same<typename Acc<T>::type, float>::value) return store_cast<T>(__builtin_nanf(""));
  else return std::numeric_limits<T>::min();
}

template <typename T, int OP>
__global__ __launch_bounds__(kThreads) void one_shot_allreduce_kernel(IO io, long n, Peers peers, int rank0, int world,
                                                                      uint32_t epoch, long slot_bytes, int* err,
                                                                      uint64_t timeout_ticks) {
  using A = typename Acc<T>::type;
  const int b = blockIdx.x, nb = gridDim.x, tid = threadIdx.x;
  const int rank = rank0 + blockIdx.y;
  const T* __restrict__ in = reinterpret_cast<const T*>(io.in[blockIdx.y]);
  T* __restrict__ out = reinterpret_cast<T*>(io.out[blockIdx.y]);
  ACC_CHECK_OR_RETURN(n * (long)sizeof(T) <= slot_bytes && rank < world, kChkAllreduceSize);  // debug build
  const long per = (n + nb - 1) / nb;
  const long lo = (long)b * per, hi = min(n, lo + per);
  const long data_off = kFlagBytes + (long)(epoch & 1) * slot_bytes;
  // 1. push this rank's chunk into its own buffer (plain stores; 16-B when aligned)
  T* mine = reinterpret_cast<T*>(peers.buf[rank] + data_off);
  constexpr int V = 16 / sizeof(T);
  const bool vec = (lo % V) == 0 && (hi % V) == 0 && ((reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out)) % 16) == 0;
  if (vec) {
    for (long i = lo + (long)tid * V; i < hi; i += (long)kThreads * V)
      *reinterpret_cast<uint4*>(mine + i) = *reinterpret_cast<const uint4*>(in + i);
  } else {
    for (long i = lo + tid; i < hi; i += kThreads) mine[i] = in[i];
  }
  // 2. release: this workgroup's data before its flag, in every peer's buffer (one lane per peer). Every lane's own
  // system-scope fence first, so the flag lanes' release covers the stores of all waves.
  __threadfence_system();
  __syncthreads();
  if (tid < world) {
    uint32_t* f = reinterpret_cast<uint32_t*>(peers.buf[tid]) + rank * kMaxBlocks + b;
    __hip_atomic_store(f, epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  // 3. acquire: wait for every peer's flag for this block in the local buffer (bounded)
  __shared__ int timed_out;
  if (tid == 0) timed_out = 0;
  __syncthreads();
  if (tid < world) {
    const uint32_t* f = reinterpret_cast<const uint32_t*>(peers.buf[rank]) + tid * kMaxBlocks + b;
    const uint64_t t0 = __builtin_amdgcn_s_memrealtime();  // 100 MHz constant clock
    while (__hip_atomic_load(f, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM) != epoch) {
      if (__builtin_amdgcn_s_memrealtime() - t0 > timeout_ticks) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
        timed_out = 1;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  if (timed_out) {
    // a peer never arrived: poison this chunk (NaN for floats, the minimum value for integers) so a caller that reads
    // the result before checking sar_status cannot consume a sum of stale peer data
    for (long i = lo + tid; i < hi; i += kThreads) out[i] = poison<T>();
    return;
  }
  __threadfence_system();
  // 4. reduce the peers' copies of the chunk (remote loads over xGMI) in registers, rank order fixed for determinism
  if (vec) {
    for (long i = lo + (long)tid * V; i < hi; i += (long)kThreads * V) {
      A acc[V];
      for (int p = 0; p < world; ++p) {
        const uint4 raw = *reinterpret_cast<const uint4*>(reinterpret_cast<const T*>(peers.buf[p] + data_off) + i);
        const T* v = reinterpret_cast<const T*>(&raw);
#pragma unroll
        for (int j = 0; j < V; ++j) {
          const A x = load_acc<T>(v + j);
          acc[j] = p == 0 ? x : (OP == kSum ? acc[j] + x : (x > acc[j] ? x : acc[j]));
        }
      }
      uint4 o;
      T* ov = reinterpret_cast<T*>(&o);
#pragma unroll
      for (int j = 0; j < V; ++j) ov[j] = store_cast<T>(acc[j]);
      *reinterpret_cast<uint4*>(out + i) = o;
    }
  } else {
    for (long i = lo + tid; i < hi; i += kThreads) {
      A acc = A(0);
      for (int p = 0; p < world; ++p) {
        const A x = load_acc<T>(reinterpret_cast<const T*>(peers.buf[p] + data_off) + i);
        acc = p == 0 ? x : (OP == kSum ? acc + x : (x > acc ? x : acc));
      }
      out[i] = store_cast<T>(acc);
    }
  }
}

struct Comm {
  int rank = 0, world = 1;
  long max_bytes = 0;
  uint8_t* local = nullptr;
  Peers peers{};
  bool opened[kMaxRanks] = {};
  uint32_t epoch = 0;
  int* err = nullptr;  // host-mapped
  int* err_dev = nullptr;
};

std::mutex g_mu;
std::map<int64_t, Comm*> g_comms;
int64_t g_next = 1;

Comm* get(int64_t id) {
  std::lock_guard<std::mutex> lk(g_mu);
  auto it = g_comms.find(id);
  TORCH_CHECK(it != g_comms.end(), "small_allreduce: unknown communicator ", id);
  return it->second;
}

void check(hipError_t e, const char* what) { TORCH_CHECK(e == hipSuccess, "small_allreduce: ", what, ": ", hipGetErrorString(e)); }

}  // namespace

ACC_DEBUG_TAKE_FN(acc_dbg_take_small_allreduce)

// Allocate this rank's buffer; returns (communicator id, IPC handle bytes of the buffer).
std::tuple<int64_t, pybind11::bytes> sar_create(int64_t rank, int64_t world, int64_t max_bytes) {
  TORCH_CHECK(world >= 1 && world <= kMaxRanks && rank >= 0 && rank < world, "small_allreduce: 1..8 ranks");
  TORCH_CHECK(max_bytes > 0 && max_bytes % 16 == 0, "small_allreduce: max_bytes must be a positive multiple of 16");
  auto* c = new Comm();
  c->rank = (int)rank;
  c->world = (int)world;
  c->max_bytes = max_bytes;
  const size_t total = kFlagBytes + 2 * (size_t)max_bytes;
  check(hipExtMallocWithFlags(reinterpret_cast<void**>(&c->local), total, hipDeviceMallocUncached), "alloc");
  check(hipMemset(c->local, 0, total), "memset");
  check(hipHostMalloc(reinterpret_cast<void**>(&c->err), sizeof(int), hipHostMallocMapped), "host alloc");
  *c->err = 0;
  check(hipHostGetDevicePointer(reinterpret_cast<void**>(&c->err_dev), c->err, 0), "host map");
  c->peers.buf[rank] = c->local;
  c->opened[rank] = false;
  hipIpcMemHandle_t h;
  check(hipIpcGetMemHandle(&h, c->local), "ipc handle");
  check(hipDeviceSynchronize(), "sync");
  int64_t id;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    id = g_next++;
    g_comms[id] = c;
  }
  return {id, pybind11::bytes(reinterpret_cast<const char*>(&h), sizeof(h))};
}

// Map the peers' buffers (handles[p] from rank p's sar_create; this rank's own entry is ignored).
void sar_open(int64_t id, std::vector<std::string> handles) {
  Comm* c = get(id);
  TORCH_CHECK((int)handles.size() == c->world, "small_allreduce: one handle per rank");
  for (int p = 0; p < c->world; ++p) {
    if (p == c->rank) continue;
    TORCH_CHECK(handles[p].size() == sizeof(hipIpcMemHandle_t), "small_allreduce: bad handle size");
    hipIpcMemHandle_t h;
    memcpy(&h, handles[p].data(), sizeof(h));
    void* ptr = nullptr;
    check(hipIpcOpenMemHandle(&ptr, h, hipIpcMemLazyEnablePeerAccess), "ipc open");
    c->peers.buf[p] = reinterpret_cast<uint8_t*>(ptr);
    c->opened[p] = true;
  }
}

// Test hook: link communicators created in ONE process (virtual peers on one GPU) without IPC.
void sar_link_local(std::vector<int64_t> ids) {
  std::vector<Comm*> cs;
  for (auto id : ids) cs.push_back(get(id));
  for (auto* c : cs) {
    TORCH_CHECK((int)cs.size() == c->world, "small_allreduce: link one communicator per rank");
    for (auto* q : cs) c->peers.buf[q->rank] = q->local;
  }
}

namespace {

void launch(Comm* c, const IO& io, int ny, int rank0, long n, at::ScalarType dt, int64_t op, double timeout_ms, long bytes) {
  const uint64_t ticks = (uint64_t)(std::max(1.0, timeout_ms) * 1e5);  // s_memrealtime runs at 100 MHz
  const int nb = (int)std::min<long>(kMaxBlocks, std::max<long>(1, (bytes + 8191) / 8192));
  auto stream = at::hip::getCurrentHIPStream();
#define SAR_LAUNCH(T, OPV)                                                                                              \
  hipLaunchKernelGGL((one_shot_allreduce_kernel<T, OPV>), dim3(nb, ny), dim3(kThreads), 0, stream, io, n, c->peers, rank0, \
                     c->world, c->epoch, c->max_bytes, c->err_dev, ticks)
#define SAR_OP(T) do { if (op == kSum) SAR_LAUNCH(T, kSum); else SAR_LAUNCH(T, kMax); } while (0)
  switch (dt) {
    case at::kFloat: SAR_OP(float); break;
    case at::kBFloat16: SAR_OP(bf16_t); break;
    case at::kLong: SAR_OP(int64_t); break;
    case at::kInt: SAR_OP(int32_t); break;
    default: TORCH_CHECK(false, "small_allreduce: dtype must be fp32, bf16, int32 or int64");
  }
#undef SAR_OP
#undef SAR_LAUNCH
}

void check_io(Comm* c, const torch::Tensor& in, const torch::Tensor& out, int64_t op) {
  TORCH_CHECK(in.is_cuda() && out.is_cuda() && in.is_contiguous() && out.is_contiguous() && in.numel() == out.numel() &&
                  in.scalar_type() == out.scalar_type(), "small_allreduce: contiguous same-shape HIP tensors");
  TORCH_CHECK(*c->err == 0, "small_allreduce: a previous call timed out waiting for a peer");
  TORCH_CHECK(in.numel() * in.element_size() <= c->max_bytes, "small_allreduce: message larger than the buffer");
  TORCH_CHECK(op == kSum || op == kMax, "small_allreduce: op must be sum or max");
}

}  // namespace

// out = reduce(in over ranks); in / out: contiguous, same dtype (fp32, bf16, int32, int64), <= max_bytes, may alias.
// op: 0 sum, 1 max. timeout_ms bounds each wait for a peer (then the call is marked failed, see sar_status).
void sar_allreduce(int64_t id, torch::Tensor in, torch::Tensor out, int64_t op, double timeout_ms) {
  Comm* c = get(id);
  check_io(c, in, out, op);
  if (in.numel() == 0) return;
  c->epoch += 1;
  IO io{};
  io.in[0] = in.data_ptr();
  io.out[0] = out.data_ptr();
  launch(c, io, 1, c->rank, in.numel(), in.scalar_type(), op, timeout_ms, in.numel() * in.element_size());
}

// Test hook: every rank of a set of communicators linked with sar_link_local, in ONE launch (virtual peers).
void sar_allreduce_local_group(std::vector<int64_t> ids, std::vector<torch::Tensor> ins, std::vector<torch::Tensor> outs,
                               int64_t op, double timeout_ms) {
  TORCH_CHECK(!ids.empty() && ids.size() == ins.size() && ids.size() == outs.size(), "small_allreduce: one in/out per rank");
  IO io{};
  Comm* c0 = get(ids[0]);
  for (size_t r = 0; r < ids.size(); ++r) {
    Comm* c = get(ids[r]);
    TORCH_CHECK(c->rank == (int)r && c->world == (int)ids.size() && c->epoch == c0->epoch, "small_allreduce: ids in rank order");
    check_io(c, ins[r], outs[r], op);
    TORCH_CHECK(ins[r].numel() == ins[0].numel() && ins[r].scalar_type() == ins[0].scalar_type(), "small_allreduce: shapes");
    io.in[r] = ins[r].data_ptr();
    io.out[r] = outs[r].data_ptr();
  }
  if (ins[0].numel() == 0) return;
  for (auto id : ids) get(id)->epoch += 1;
  launch(c0, io, (int)ids.size(), 0, ins[0].numel(), ins[0].scalar_type(), op, timeout_ms, ins[0].numel() * ins[0].element_size());
}

// 0 = healthy, 1 = a wait timed out (the results of that call are invalid).
int64_t sar_status(int64_t id) { return *get(id)->err; }

void sar_destroy(int64_t id) {
  Comm* c;
  {
    std::lock_guard<std::mutex> lk(g_mu);
    auto it = g_comms.find(id);
    if (it == g_comms.end()) return;
    c = it->second;
    g_comms.erase(it);
  }
  hipDeviceSynchronize();
  for (int p = 0; p < c->world; ++p)
    if (c->opened[p]) hipIpcCloseMemHandle(c->peers.buf[p]);
  hipFree(c->local);
  hipHostFree(c->err);
  delete c;
}
