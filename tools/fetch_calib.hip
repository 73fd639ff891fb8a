// FETCH_SIZE / WRITE_SIZE calibration on a known byte count (MI355X_MICROARCH.md,
// HBM section: "Other access widths are uncalibrated: calibrate on a known
// byte count in your own access pattern").
//
// Streams a 1 GiB buffer (4x the 256 MiB Infinity Cache, so every launch goes
// to HBM) with 4-, 8- and 16-byte lane loads (coalesced, grid-strided: the
// access shapes of the SELL word stream, the real(8) and the complex(8)
// vector streams), and writes it with the same widths.  Run under
// `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` (separate passes);
// counter / bytes gives the correction factor per width.
//
// build: hipcc -O3 --offload-arch=gfx950 -o tools/fetch_calib tools/fetch_calib.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x)                                                                    \
  do {                                                                           \
    hipError_t e_ = (x);                                                         \
    if (e_ != hipSuccess) {                                                      \
      fprintf(stderr, "%s -> %s\n", #x, hipGetErrorString(e_));                  \
      return 1;                                                                  \
    }                                                                            \
  } while (0)

__device__ __forceinline__ uint32_t fold(uint32_t v) { return v; }
__device__ __forceinline__ uint32_t fold(uint2 v) { return v.x ^ v.y; }
__device__ __forceinline__ uint32_t fold(uint4 v) { return v.x ^ v.y ^ v.z ^ v.w; }
template <class T> __device__ __forceinline__ T mkv(uint32_t s);
template <> __device__ __forceinline__ uint32_t mkv<uint32_t>(uint32_t s) { return s; }
template <> __device__ __forceinline__ uint2 mkv<uint2>(uint32_t s) { return make_uint2(s, s + 1); }
template <> __device__ __forceinline__ uint4 mkv<uint4>(uint32_t s) { return make_uint4(s, s + 1, s + 2, s + 3); }

// read n elements of T; one word per block so the loads cannot be elided
template <class T>
__global__ void __launch_bounds__(256) k_read(const T* __restrict__ p, int64_t n, uint32_t* __restrict__ out) {
  uint32_t acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) acc ^= fold(p[i]);
  if (acc == 0x9e3779b9u) out[blockIdx.x] = acc;  // practically never: no write traffic
}

template <class T>
__global__ void __launch_bounds__(256) k_write(T* __restrict__ p, int64_t n, uint32_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256)
    p[i] = mkv<T>(seed ^ (uint32_t)i);
}

template <class T>
static int run(const char* name, void* buf, size_t bytes, uint32_t* out, int iters) {
  const int64_t n = (int64_t)(bytes / sizeof(T));
  const int grid = 256 * 16;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int w = 0; w < 2; w++) {
    CK(hipEventRecord(e0, 0));
    for (int i = 0; i < iters; i++) {
      if (w == 0) hipLaunchKernelGGL(k_read<T>, dim3(grid), dim3(256), 0, 0, (const T*)buf, n, out);
      else hipLaunchKernelGGL(k_write<T>, dim3(grid), dim3(256), 0, 0, (T*)buf, n, (uint32_t)i);
    }
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= iters;
    printf("%s %s: %zu bytes/launch, %.4f ms, %.1f GB/s\n", w ? "write" : "read", name, bytes, ms,
           bytes / (ms * 1e-3) / 1e9);
  }
  CK(hipEventDestroy(e0));
  CK(hipEventDestroy(e1));
  return 0;
}

int main() {
  const size_t bytes = (size_t)1 << 30;
  void* buf;
  uint32_t* out;
  CK(hipMalloc(&buf, bytes));
  CK(hipMalloc((void**)&out, 1 << 20));
  CK(hipMemset(buf, 1, bytes));
  if (run<uint32_t>("b32", buf, bytes, out, 5)) return 1;
  if (run<uint2>("b64", buf, bytes, out, 5)) return 1;
  if (run<uint4>("b128", buf, bytes, out, 5)) return 1;
  CK(hipDeviceSynchronize());
  CK(hipFree(buf));
  CK(hipFree(out));
  printf("CALIB_DONE\n");
  return 0;
}
