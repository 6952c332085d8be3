// Cost of a device-wide barrier inside one persistent kernel against a kernel boundary, for the
// nested-sampling generation (walk -> merge -> walk ...).  Both forms run the same two phases per
// iteration (phase 1 writes a 1 MB buffer, phase 2 reads it back and writes another) over
// 256 workgroups of 256 threads (one per CU):
//   kernels:    2 launches per iteration, stream-ordered
//   persistent: one launch, a grid barrier after each phase (agent-scope atomic counter, release /
//               acquire fences), every wait bounded (a workgroup that waits too long sets an error
//               flag and leaves, so the grid always drains)
//   hipcc --offload-arch=gfx950 -O3 grid_barrier.hip -o /tmp/grid_barrier && /tmp/grid_barrier
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

constexpr int kBlocks = 256, kThreads = 256;
constexpr int kElems = 1 << 17;          // 1 MB of doubles

__global__ void phase1(double* a, const double* b, int it) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kElems; i += gridDim.x * blockDim.x)
    a[i] = b[(i * 7 + it) & (kElems - 1)] + 1.0;
}
__global__ void phase2(double* b, const double* a, int it) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kElems; i += gridDim.x * blockDim.x)
    b[i] = a[(i * 13 + it) & (kElems - 1)] * 0.5;
}

__device__ bool grid_barrier(unsigned* ctr, unsigned target, int* err) {
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    long guard = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++guard > (1L << 24)) { __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); ok = false; break; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __shared__ int s_ok;
  if (threadIdx.x == 0) s_ok = ok;
  __syncthreads();
  return s_ok;
}

// the same barrier polling with relaxed loads (no cache invalidate per poll), one acquire fence
// once the count is reached
__device__ bool grid_barrier_relaxed(unsigned* ctr, unsigned target, int* err) {
  __syncthreads();
  bool ok = true;
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    long guard = 0;
    while (__hip_atomic_load(ctr, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (++guard > (1L << 24)) { __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); ok = false; break; }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  __shared__ int s_ok;
  if (threadIdx.x == 0) s_ok = ok;
  __syncthreads();
  return s_ok;
}

__global__ void persistent_relaxed(double* a, double* b, int iters, unsigned* ctr, int* err) {
  unsigned target = 0;
  for (int it = 0; it < iters; ++it) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kElems; i += gridDim.x * blockDim.x)
      a[i] = b[(i * 7 + it) & (kElems - 1)] + 1.0;
    target += gridDim.x;
    if (!grid_barrier_relaxed(ctr, target, err)) return;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kElems; i += gridDim.x * blockDim.x)
      b[i] = a[(i * 13 + it) & (kElems - 1)] * 0.5;
    target += gridDim.x;
    if (!grid_barrier_relaxed(ctr, target, err)) return;
  }
}

__global__ void persistent(double* a, double* b, int iters, unsigned* ctr, int* err) {
  unsigned target = 0;
  for (int it = 0; it < iters; ++it) {
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kElems; i += gridDim.x * blockDim.x)
      a[i] = b[(i * 7 + it) & (kElems - 1)] + 1.0;
    target += gridDim.x;
    if (!grid_barrier(ctr, target, err)) return;
    for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < kElems; i += gridDim.x * blockDim.x)
      b[i] = a[(i * 13 + it) & (kElems - 1)] * 0.5;
    target += gridDim.x;
    if (!grid_barrier(ctr, target, err)) return;
  }
}

int main() {
  int ncu = 0, occ = 0;
  HC(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  HC(hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, persistent, kThreads, 0));
  printf("CUs %d, resident blocks per CU %d\n", ncu, occ);
  if (ncu * occ < kBlocks) { printf("grid not co-resident: skip\n"); return 0; }
  double *a, *b;
  unsigned* ctr;
  int* err;
  HC(hipMalloc(&a, kElems * 8));
  HC(hipMalloc(&b, kElems * 8));
  HC(hipMalloc(&ctr, 4));
  HC(hipMalloc(&err, 4));
  HC(hipMemset(a, 0, kElems * 8));
  HC(hipMemset(b, 0, kElems * 8));
  hipEvent_t e0, e1;
  HC(hipEventCreate(&e0));
  HC(hipEventCreate(&e1));
  const int iters = 1000;
  for (int rep = 0; rep < 3; ++rep) {
    HC(hipEventRecord(e0, 0));
    for (int it = 0; it < iters; ++it) {
      phase1<<<kBlocks, kThreads>>>(a, b, it);
      phase2<<<kBlocks, kThreads>>>(b, a, it);
    }
    HC(hipEventRecord(e1, 0));
    HC(hipEventSynchronize(e1));
    float ms = 0;
    HC(hipEventElapsedTime(&ms, e0, e1));
    printf("kernels:    %.2f us per iteration (2 launches)\n", 1000.0 * ms / iters);
    HC(hipMemset(ctr, 0, 4));
    HC(hipMemset(err, 0, 4));
    HC(hipEventRecord(e0, 0));
    persistent<<<kBlocks, kThreads>>>(a, b, iters, ctr, err);
    HC(hipEventRecord(e1, 0));
    HC(hipEventSynchronize(e1));
    HC(hipEventElapsedTime(&ms, e0, e1));
    int herr = 0;
    HC(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    printf("persistent: %.2f us per iteration (2 grid barriers)%s\n", 1000.0 * ms / iters, herr ? "  [barrier timeout]" : "");
    HC(hipMemset(ctr, 0, 4));
    HC(hipMemset(err, 0, 4));
    HC(hipEventRecord(e0, 0));
    persistent_relaxed<<<kBlocks, kThreads>>>(a, b, iters, ctr, err);
    HC(hipEventRecord(e1, 0));
    HC(hipEventSynchronize(e1));
    HC(hipEventElapsedTime(&ms, e0, e1));
    HC(hipMemcpy(&herr, err, 4, hipMemcpyDeviceToHost));
    printf("relaxed:    %.2f us per iteration (2 grid barriers, relaxed polling)%s\n", 1000.0 * ms / iters, herr ? "  [barrier timeout]" : "");
  }
  return 0;
}
