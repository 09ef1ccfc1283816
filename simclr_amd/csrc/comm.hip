// One-shot IPC collectives for the gathered NT-Xent: the bf16 embedding
// all-gather of the forward and the fp32 column-gradient reduce-scatter of the backward, over
// the same peer-mapped uncached arenas and LL-word protocol as the BatchNorm statistics exchange
// (bn.hip bn_ipc_exchange, comm/ipc.py): every 8-byte word carries 4 payload bytes in its low
// half and the exchange epoch in its high half, so ONE vector store publishes data and flag
// (no fences, no L2 write-back), and a reader spins until every word it needs shows the epoch.
//
// Site layout (int64 words, the same offset in every rank's arena): 2 parities x W rank slots
// x n words; exchange e uses parity e & 1 (a rank can only start exchange e + 2 after it — and
// therefore every peer — finished reading exchange e, so a slot is never overwritten early).
// Each block owns a fixed chunk of the n words and its own epoch counter (one writer per
// counter, no atomics); the grid size is fixed per site (host: IPC_COLL_BLOCKS).
//
// Spins are wall-clock bounded (2 s, then the sticky error flag, as in bn.hip): a lost peer
// costs seconds and an IpcExchangeError at the next step check, never a hung GPU.
//
//   ipc_allgather: dst[r][i] = src_r[i] for every rank r (32-bit words: bf16 pairs)
//   ipc_reduce_scatter: dst[i] = sum_r src_r[rank * n + i] in rank order — bitwise identical
//                       whichever rank computes it (each rank sums only its own slice)
#include "common.h"
#include "kernels.h"

namespace {

constexpr int kCollMaxWorld = 16;
constexpr long long kSpinNs10 = 200000000LL;  // 2 s of the 100 MHz constant clock

struct IpcCollArgs {
  const uint32_t* src;       // allgather: [n] own words; reduce_scatter: [W][n] fp32 bits
  uint32_t* dst;             // allgather: [W][n]; reduce_scatter: [n]
  uint64_t* const* peers;    // [W] arena bases (own included)
  uint64_t* own;
  long long site;            // word offset of the site region (2 x W x n words)
  unsigned* epoch;           // [gridDim.x] per-block exchange counters
  int* err;
  int n, W, rank, chunk;
};

__device__ __forceinline__ unsigned next_epoch(const IpcCollArgs& p, unsigned* sh) {
  if (threadIdx.x == 0) {
    const unsigned e = p.epoch[blockIdx.x] + 1u;
    p.epoch[blockIdx.x] = e;
    *sh = e;
  }
  __syncthreads();
  return *sh;
}

// spin until the word at `src` carries epoch e; returns its payload (0 after a timeout)
__device__ __forceinline__ uint32_t ll_wait(const uint64_t* src, unsigned e, long long t0,
                                            bool& dead, int* err) {
  uint64_t w = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  while ((unsigned)(w >> 32) != e) {
    if (dead || (long long)wall_clock64() - t0 > kSpinNs10) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      dead = true;
      return 0u;
    }
    __builtin_amdgcn_s_sleep(1);
    w = __hip_atomic_load(src, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  }
  return (uint32_t)w;
}

__global__ __launch_bounds__(256) void k_ipc_allgather(IpcCollArgs p) {
  __shared__ unsigned sh_e;
  const unsigned e = next_epoch(p, &sh_e);
  const long long slot = p.n;
  const long long base = p.site + (long long)(e & 1u) * p.W * slot;
  const int i0 = blockIdx.x * p.chunk;
  const int i1 = min(p.n, i0 + p.chunk);
  // push this rank's chunk into slot `rank` of every arena (its own included)
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    const uint64_t w = ((uint64_t)e << 32) | (uint64_t)p.src[i];
    for (int r = 0; r < p.W; ++r)
      __hip_atomic_store(p.peers[r] + base + (long long)p.rank * slot + i, w, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
  const long long t0 = (long long)wall_clock64();
  bool dead = __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  for (int r = 0; r < p.W; ++r)
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x)
      p.dst[(long long)r * p.n + i] = ll_wait(p.own + base + (long long)r * slot + i, e, t0, dead,
                                              p.err);
}

__global__ __launch_bounds__(256) void k_ipc_reduce_scatter(IpcCollArgs p) {
  __shared__ unsigned sh_e;
  const unsigned e = next_epoch(p, &sh_e);
  const long long slot = p.n;
  const long long base = p.site + (long long)(e & 1u) * p.W * slot;
  const int i0 = blockIdx.x * p.chunk;
  const int i1 = min(p.n, i0 + p.chunk);
  // push peer r's slice of this rank's full gradient into slot `rank` of r's arena
  for (int r = 0; r < p.W; ++r)
    for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
      const uint64_t w = ((uint64_t)e << 32) | (uint64_t)p.src[(long long)r * p.n + i];
      __hip_atomic_store(p.peers[r] + base + (long long)p.rank * slot + i, w, __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
    }
  const long long t0 = (long long)wall_clock64();
  bool dead = __hip_atomic_load(p.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0;
  for (int i = i0 + threadIdx.x; i < i1; i += blockDim.x) {
    float a = 0.f;
    for (int r = 0; r < p.W; ++r)  // rank order: the same sum on every rank
      a += __uint_as_float(ll_wait(p.own + base + (long long)r * slot + i, e, t0, dead, p.err));
    p.dst[i] = __float_as_uint(a);
  }
}

}  // namespace

long long ipc_coll_region_words(int world, int n) { return 2LL * world * n; }

void ipc_collective(int op, const uint32_t* src, uint32_t* dst, int n, uint64_t* const* peers,
                    uint64_t* own, long long site, unsigned* epoch, int* err, int world,
                    int rank, hipStream_t s) {
  IpcCollArgs a{};
  a.src = src; a.dst = dst; a.peers = peers; a.own = own; a.site = site; a.epoch = epoch;
  a.err = err; a.n = n; a.W = world; a.rank = rank;
  a.chunk = (n + IPC_COLL_BLOCKS - 1) / IPC_COLL_BLOCKS;
  if (op == 0)
    hipLaunchKernelGGL(k_ipc_allgather, dim3(IPC_COLL_BLOCKS), dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(k_ipc_reduce_scatter, dim3(IPC_COLL_BLOCKS), dim3(256), 0, s, a);
  HIP_CHECK_LAUNCH();
}
