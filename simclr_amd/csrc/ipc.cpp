// Peer-mapped device memory for the one-shot statistics exchange (bn.hip bn_ipc_exchange).
//
// Each rank allocates ONE arena of fine-grained, uncached device memory (remote 64-bit stores
// from peers land in HBM and the local spinning loads never hit a stale L2 line), exports it
// with hipIpcGetMemHandle, and maps every peer's arena with hipIpcOpenMemHandle (peer access
// over xGMI enabled lazily by the runtime).  The handles travel through the process group's
// object all-gather (simclr_amd/comm/ipc.py); the kernels get a device table of the W bases.
#include <ATen/core/Tensor.h>
#include <ATen/ops/empty.h>
#include <ATen/ops/from_blob.h>
#include <ATen/hip/HIPContext.h>
#include <c10/util/Exception.h>
#include <hip/hip_runtime.h>
#include <torch/library.h>

#include <cstring>

using at::Tensor;

namespace {

#define IPC_CHECK(expr)                                                                  \
  do {                                                                                   \
    hipError_t e_ = (expr);                                                              \
    TORCH_CHECK(e_ == hipSuccess, #expr " failed: ", hipGetErrorString(e_));             \
  } while (0)

// int64 words, zeroed (epoch 0 never matches a live exchange: epochs start at 1)
Tensor ipc_arena_alloc(int64_t words, int64_t device) {
  TORCH_CHECK(words > 0, "ipc_arena_alloc: size");
  int prev = 0;
  IPC_CHECK(hipGetDevice(&prev));
  IPC_CHECK(hipSetDevice((int)device));
  void* p = nullptr;
  IPC_CHECK(hipExtMallocWithFlags(&p, (size_t)words * 8, hipDeviceMallocUncached));
  IPC_CHECK(hipMemset(p, 0, (size_t)words * 8));
  IPC_CHECK(hipDeviceSynchronize());
  IPC_CHECK(hipSetDevice(prev));
  auto opts = at::TensorOptions().dtype(at::kLong).device(at::Device(at::kCUDA, (int)device));
  return at::from_blob(p, {words}, [](void* q) { (void)hipFree(q); }, opts);
}

Tensor ipc_handle(const Tensor& arena) {
  TORCH_CHECK(arena.is_cuda(), "ipc_handle: GPU arena expected");
  hipIpcMemHandle_t h;
  IPC_CHECK(hipIpcGetMemHandle(&h, arena.data_ptr()));
  Tensor out = at::empty({(int64_t)sizeof(h)}, at::TensorOptions().dtype(at::kByte));
  std::memcpy(out.data_ptr(), &h, sizeof(h));
  return out;
}

// maps a peer's arena into this process; returns the device address (kept open for the life of
// the process group, closed by ipc_close)
int64_t ipc_open(const Tensor& handle, int64_t device) {
  hipIpcMemHandle_t h;
  TORCH_CHECK(handle.numel() == (int64_t)sizeof(h) && handle.scalar_type() == at::kByte &&
                  !handle.is_cuda(), "ipc_open: expected a CPU uint8 handle of ", sizeof(h), " bytes");
  std::memcpy(&h, handle.contiguous().data_ptr(), sizeof(h));
  int prev = 0;
  IPC_CHECK(hipGetDevice(&prev));
  IPC_CHECK(hipSetDevice((int)device));
  void* p = nullptr;
  IPC_CHECK(hipIpcOpenMemHandle(&p, h, hipIpcMemLazyEnablePeerAccess));
  IPC_CHECK(hipSetDevice(prev));
  return reinterpret_cast<int64_t>(p);
}

void ipc_close(int64_t ptr) {
  if (ptr != 0) IPC_CHECK(hipIpcCloseMemHandle(reinterpret_cast<void*>(ptr)));
}

}  // namespace

TORCH_LIBRARY_FRAGMENT(simclr_amd, m) {
  m.def("ipc_arena_alloc(int words, int device) -> Tensor", &ipc_arena_alloc);
  m.def("ipc_handle(Tensor arena) -> Tensor", &ipc_handle);
  m.def("ipc_open(Tensor handle, int device) -> int", &ipc_open);
  m.def("ipc_close(int ptr) -> ()", &ipc_close);
}
