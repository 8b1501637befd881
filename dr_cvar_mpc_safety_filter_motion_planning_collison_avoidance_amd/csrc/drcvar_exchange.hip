// drcvar_exchange.hip — the peer-push record exchange across the GPUs of one node
// (include/drcvar_exchange.h).
//
// The halfspace launch of every rank (drcvar_safe_halfspaces_f64_peer, drcvar_halfspace.hip)
// already wrote its records into every rank's region; what is left per step is one small launch:
//
//   publish   workgroup 0, lane j < n_ranks: flag[rank] of rank j's region <- g (system-scope
//             store; the halfspace launch before it on the stream has completed, and each of its
//             writing waves waited for the acknowledgement of its system-scope record stores
//             before it ended, so every record is in every region)
//   wait      every workgroup, lane j < n_ranks: poll flag[j] of the own region until >= g
//             (system-scope loads of uncached memory: no cache can hold a stale flag), bounded by
//             the 100 MHz realtime clock; a timeout sets the error word instead of hanging
//   copy      every workgroup copies its slice of the gathered parity buffer into `out` (16-B
//             nontemporal loads, which bypass L1, of the uncached region, which no L2 holds;
//             ordinary stores)
//   advance   the last workgroup to finish (a launch counter: every workgroup read the generation
//             before it counted itself) resets the counter and stores the new generation
// No cache-maintenance fence is needed on either side (each costs ~1.7 us on gfx950): the records
// and flags live in uncached memory and move by system-scope / nontemporal accesses only, and the
// generation and counter are read and written by atomics or across kernel boundaries.
//
// The grid is at most 256 workgroups of 256 threads (one per 4 K records); no workgroup waits on
// another of the launch (each polls the flags itself), so residency does not matter.
//
// The pull form (drcvar_peer_signal_wait_pull): the halfspace launch wrote its records into its
// own region only (drcvar_safe_halfspaces_f64_peer with the one-rank set {own region}: its waves
// wait for local acknowledgements, not for a write round trip over xGMI per unit); this launch
// publishes the same way, waits the same way, and copies rank j's rows of the parity buffer from
// rank j's region (nontemporal 16-B loads over xGMI).  Double buffering holds as in the push form:
// a rank rewrites parity p two steps later, after every peer has published the step in between,
// which each does only after its copy of parity p has completed (the previous launch on its
// stream).
#include <hip/hip_runtime.h>

#include <cstdint>

#include "drcvar_exchange.h"
#include "drcvar_halfspace.h"

namespace {

constexpr int kThreads = 256;
constexpr int kPerThread = 4;         // 16-B copies per thread, their loads issued together
constexpr int64_t kMaxGroups = 256;   // C5 (12 800 records, 819 KB): 50 workgroups, one pass
constexpr int64_t kFlagsDoubles = 64;  // the flag slot of a region (512 B: room for 64 ranks)
typedef double dbl2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ unsigned long long* flags_of(double* region, int64_t rows) {
  return reinterpret_cast<unsigned long long*>(region + 2 * rows * DRCVAR_OUT_WIDTH);
}

// n2 16-B elements src -> dst by the whole grid, kPerThread loads in flight per thread per pass
// (the uncached region answers from HBM: one round trip per pass, not per element)
__device__ __forceinline__ void copy_block(const dbl2* __restrict__ src, dbl2* __restrict__ dst, int64_t n2) {
  const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
  for (int64_t i0 = static_cast<int64_t>(blockIdx.x) * kThreads + threadIdx.x; i0 < n2;
       i0 += stride * kPerThread) {
    dbl2 v[kPerThread];
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) {
      const int64_t i = i0 + k * stride;
      if (i < n2) v[k] = __builtin_nontemporal_load(src + i);
    }
#pragma unroll
    for (int k = 0; k < kPerThread; ++k) {
      const int64_t i = i0 + k * stride;
      if (i < n2) dst[i] = v[k];
    }
  }
}

template <bool kPull>
__global__ void __launch_bounds__(kThreads)
peer_signal_wait_kernel(drcvar_peer_set ps, double* __restrict__ out, long long spin_ticks) {
  const int tid = threadIdx.x;
  unsigned long long* state = ps.state;
  // the generation this step completes (the previous step's launch stored the last one; this
  // launch advances it only after every workgroup has read it)
  const unsigned long long g = __hip_atomic_load(state, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) + 1ull;
  const int64_t parity = static_cast<int64_t>(g & 1ull);
  if (blockIdx.x == 0 && tid < ps.n_ranks) {  // publish: this rank's rows are in every region (pull: in its own)
    __hip_atomic_store(flags_of(ps.region[tid], ps.rows) + ps.rank, g, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  }
  if (tid < ps.n_ranks) {  // wait: every rank's rows of this parity are in the own region
    const unsigned long long* f = flags_of(ps.region[ps.rank], ps.rows) + tid;
    const long long t0 = static_cast<long long>(__builtin_amdgcn_s_memrealtime());
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < g) {
      if (static_cast<long long>(__builtin_amdgcn_s_memrealtime()) - t0 > spin_ticks) {
        __hip_atomic_fetch_or(state + 2, (1ull << 63) | (1ull << tid), __ATOMIC_RELAXED,
                              __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
  }
  __syncthreads();
  // copy: the gathered parity buffer -> out (pull: rank j's rows from rank j's region)
  dbl2* dst = reinterpret_cast<dbl2*>(out);
  if constexpr (!kPull) {
    copy_block(reinterpret_cast<const dbl2*>(ps.region[ps.rank] + parity * ps.rows * DRCVAR_OUT_WIDTH),
               dst, ps.rows * DRCVAR_OUT_WIDTH / 2);
  } else {
    // every rank's block in ONE pass, the loads of a thread (from any peers) issued together: a
    // pass per peer would put one xGMI round trip per peer in series
    const int64_t per2 = ps.rows / ps.n_ranks * (DRCVAR_OUT_WIDTH / 2);  // (host-checked: rows = n_ranks * per)
    const int64_t n2 = ps.rows * (DRCVAR_OUT_WIDTH / 2), base = parity * n2;
    const int64_t stride = static_cast<int64_t>(gridDim.x) * kThreads;
    for (int64_t i0 = static_cast<int64_t>(blockIdx.x) * kThreads + tid; i0 < n2; i0 += stride * kPerThread) {
      dbl2 v[kPerThread];
#pragma unroll
      for (int k = 0; k < kPerThread; ++k) {
        const int64_t i = i0 + k * stride;
        if (i < n2) {
          int j = 0;
          while (j + 1 < ps.n_ranks && i >= (j + 1) * per2) ++j;  // the rank whose block holds i
          v[k] = __builtin_nontemporal_load(reinterpret_cast<const dbl2*>(ps.region[j]) + base + i);
        }
      }
#pragma unroll
      for (int k = 0; k < kPerThread; ++k) {
        const int64_t i = i0 + k * stride;
        if (i < n2) dst[i] = v[k];
      }
    }
  }
  // advance: the last workgroup out stores the generation
  __syncthreads();
  if (tid == 0) {  // (g was read before this add: the poll loop above depends on its value)
    const unsigned long long done = __hip_atomic_fetch_add(state + 1, 1ull, __ATOMIC_RELAXED,
                                                           __HIP_MEMORY_SCOPE_AGENT);
    if (done + 1ull == gridDim.x) {
      __hip_atomic_store(state + 1, 0ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(state, g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

bool valid(const drcvar_peer_set* ps) {
  if (!ps || ps->n_ranks < 1 || ps->n_ranks > DRCVAR_MAX_PEERS || ps->rank < 0 ||
      ps->rank >= ps->n_ranks || ps->rows < 0 || !ps->state)
    return false;
  for (int j = 0; j < ps->n_ranks; ++j)
    if (!ps->region[j]) return false;
  return true;
}

template <bool kPull>
int signal_wait(const drcvar_peer_set* peers, double* out, int64_t spin_limit_us, void* stream) {
  if (!valid(peers) || !out || spin_limit_us <= 0) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (kPull && peers->rows % peers->n_ranks != 0) return DRCVAR_ERR_INVALID_ARGUMENT;
  const int64_t n2 = peers->rows * DRCVAR_OUT_WIDTH / 2;
  int64_t groups = (n2 + kThreads * kPerThread - 1) / (kThreads * kPerThread);
  groups = groups < 1 ? 1 : (groups > kMaxGroups ? kMaxGroups : groups);
  (void)hipGetLastError();
  hipLaunchKernelGGL(peer_signal_wait_kernel<kPull>, dim3(static_cast<unsigned>(groups)), dim3(kThreads), 0,
                     static_cast<hipStream_t>(stream), *peers, out,
                     static_cast<long long>(spin_limit_us) * 100);  // 100 MHz realtime clock
  return hipGetLastError() == hipSuccess ? DRCVAR_OK : DRCVAR_ERR_LAUNCH;
}

}  // namespace

extern "C" {

int64_t drcvar_peer_region_doubles(int64_t rows) {
  return rows < 0 ? -1 : 2 * rows * DRCVAR_OUT_WIDTH + kFlagsDoubles;
}

int drcvar_peer_alloc(int64_t doubles, double** region, void* handle_out) {
  if (doubles <= 0 || !region || !handle_out) return DRCVAR_ERR_INVALID_ARGUMENT;
  void* p = nullptr;
  const size_t bytes = static_cast<size_t>(doubles) * sizeof(double);
  if (hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached) != hipSuccess) return DRCVAR_ERR_LAUNCH;
  hipIpcMemHandle_t h;
  if (hipMemset(p, 0, bytes) != hipSuccess || hipDeviceSynchronize() != hipSuccess ||
      hipIpcGetMemHandle(&h, p) != hipSuccess) {
    (void)hipFree(p);
    return DRCVAR_ERR_LAUNCH;
  }
  static_assert(sizeof(h) == DRCVAR_PEER_HANDLE_BYTES, "IPC handle size");
  __builtin_memcpy(handle_out, &h, sizeof(h));
  *region = static_cast<double*>(p);
  return DRCVAR_OK;
}

int drcvar_peer_free(double* region) {
  if (!region) return DRCVAR_ERR_INVALID_ARGUMENT;
  return hipFree(region) == hipSuccess ? DRCVAR_OK : DRCVAR_ERR_LAUNCH;
}

int drcvar_peer_open(const void* handle, double** region) {
  if (!handle || !region) return DRCVAR_ERR_INVALID_ARGUMENT;
  hipIpcMemHandle_t h;
  __builtin_memcpy(&h, handle, sizeof(h));
  void* p = nullptr;
  if (hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess) != hipSuccess || !p)
    return DRCVAR_ERR_LAUNCH;
  *region = static_cast<double*>(p);
  return DRCVAR_OK;
}

int drcvar_peer_close(double* region) {
  if (!region) return DRCVAR_ERR_INVALID_ARGUMENT;
  return hipIpcCloseMemHandle(region) == hipSuccess ? DRCVAR_OK : DRCVAR_ERR_LAUNCH;
}

int drcvar_peer_can_access(int32_t device, int32_t peer_device, int32_t* can_access) {
  if (!can_access || device < 0 || peer_device < 0) return DRCVAR_ERR_INVALID_ARGUMENT;
  if (device == peer_device) {
    *can_access = 1;
    return DRCVAR_OK;
  }
  int c = 0;
  if (hipDeviceCanAccessPeer(&c, device, peer_device) != hipSuccess) return DRCVAR_ERR_LAUNCH;
  *can_access = c ? 1 : 0;
  return DRCVAR_OK;
}

int drcvar_peer_bus_id(int32_t device, char* bus_id, int32_t len) {
  if (!bus_id || len < 13 || device < 0) return DRCVAR_ERR_INVALID_ARGUMENT;
  return hipDeviceGetPCIBusId(bus_id, len, device) == hipSuccess ? DRCVAR_OK : DRCVAR_ERR_LAUNCH;
}

int drcvar_peer_device_of(const char* bus_id, int32_t* device) {
  if (!bus_id || !device) return DRCVAR_ERR_INVALID_ARGUMENT;
  int d = -1;
  if (hipDeviceGetByPCIBusId(&d, bus_id) != hipSuccess || d < 0) return DRCVAR_ERR_UNSUPPORTED;
  *device = d;
  return DRCVAR_OK;
}


int drcvar_peer_signal_wait(const drcvar_peer_set* peers, double* out, int64_t spin_limit_us,
                            void* stream) {
  return signal_wait<false>(peers, out, spin_limit_us, stream);
}

int drcvar_peer_signal_wait_pull(const drcvar_peer_set* peers, double* out, int64_t spin_limit_us,
                                 void* stream) {
  return signal_wait<true>(peers, out, spin_limit_us, stream);
}

}  // extern "C"
