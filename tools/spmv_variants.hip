// spmv_variants.hip — A/B timing of SELL-64 SpMV kernel variants on the real
// Nlevels=28 (7,7) sector matrix built by libedgpu.so (experiment tool, not
// part of the product).  Every variant must reproduce the library's k_spmv
// result bit for bit.
//
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off \
//          -I../include tools/spmv_variants.hip -L dmft-ed_amd -ledgpu -o tools/spmv_variants
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "../include/ed_gpu.h"

#define CK(x)                                                             \
  do {                                                                    \
    hipError_t e = (x);                                                   \
    if (e != hipSuccess) {                                                \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                            \
    }                                                                     \
  } while (0)

template <int NT>
__device__ __forceinline__ double ldv(const double* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int NT>
__device__ __forceinline__ int ldc(const int* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}

// V0: baseline generic (as the library)
template <int BS>
__global__ void __launch_bounds__(BS) v0(const double* __restrict__ diag, const int64_t* __restrict__ sptr,
                                         const int* __restrict__ cols, const double* __restrict__ vals,
                                         const double* __restrict__ x, double* __restrict__ y, int64_t dim,
                                         int64_t nslice) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < nslice * 64; i += (int64_t)gridDim.x * BS) {
    if (i < dim) {
      int64_t s = i >> 6, s0 = sptr[s];
      int w = (int)((sptr[s + 1] - s0) >> 6);
      int64_t base = s0 + (i & 63);
      double acc = 0.0 + diag[i] * x[i];
#pragma unroll 4
      for (int k = 0; k < w; k++) {
        int64_t q = base + 64 * (int64_t)k;
        acc = acc + vals[q] * x[cols[q]];
      }
      y[i] = acc;
    }
  }
}

// V1: chunks of C entries, loads of a chunk issued before use; NT = nontemporal matrix loads
template <int BS, int C, int NT>
__global__ void __launch_bounds__(BS) v1(const double* __restrict__ diag, const int64_t* __restrict__ sptr,
                                         const int* __restrict__ cols, const double* __restrict__ vals,
                                         const double* __restrict__ x, double* __restrict__ y, int64_t dim,
                                         int64_t nslice) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < nslice * 64; i += (int64_t)gridDim.x * BS) {
    if (i < dim) {
      int64_t s = i >> 6, s0 = sptr[s];
      int w = (int)((sptr[s + 1] - s0) >> 6);
      const int* cp = cols + s0 + (i & 63);
      const double* vp = vals + s0 + (i & 63);
      double acc = 0.0 + ldv<NT>(diag + i) * x[i];
      for (int k0 = 0; k0 < w; k0 += C) {
        int c[C];
        double h[C], g[C];
#pragma unroll
        for (int k = 0; k < C; k++) c[k] = (k0 + k < w) ? ldc<NT>(cp + 64 * (k0 + k)) : (int)i;
#pragma unroll
        for (int k = 0; k < C; k++) h[k] = (k0 + k < w) ? ldv<NT>(vp + 64 * (k0 + k)) : 0.0;
#pragma unroll
        for (int k = 0; k < C; k++) g[k] = x[c[k]];
#pragma unroll
        for (int k = 0; k < C; k++)
          if (k0 + k < w) acc = acc + h[k] * g[k];
      }
      y[i] = acc;
    }
  }
}

// V3: compile-time width W (uniform-width matrices)
template <int BS, int W, int NT>
__global__ void __launch_bounds__(BS) v3(const double* __restrict__ diag, const int64_t* __restrict__ sptr,
                                         const int* __restrict__ cols, const double* __restrict__ vals,
                                         const double* __restrict__ x, double* __restrict__ y, int64_t dim,
                                         int64_t nslice) {
  for (int64_t i = (int64_t)blockIdx.x * BS + threadIdx.x; i < nslice * 64; i += (int64_t)gridDim.x * BS) {
    if (i < dim) {
      int64_t s0 = sptr[i >> 6];
      const int* cp = cols + s0 + (i & 63);
      const double* vp = vals + s0 + (i & 63);
      int c[W];
      double h[W];
#pragma unroll
      for (int k = 0; k < W; k++) c[k] = ldc<NT>(cp + 64 * k);
#pragma unroll
      for (int k = 0; k < W; k++) h[k] = ldv<NT>(vp + 64 * k);
      double acc = 0.0 + ldv<NT>(diag + i) * x[i];
#pragma unroll
      for (int k = 0; k < W; k++) acc = acc + h[k] * x[c[k]];
      y[i] = acc;
    }
  }
}

typedef void (*kfn)(const double*, const int64_t*, const int*, const double*, const double*, double*,
                    int64_t, int64_t);

int main(int argc, char** argv) {
  int norb = argc > 1 ? atoi(argv[1]) : 1;
  int nbath = argc > 2 ? atoi(argv[2]) : 13;
  int q = argc > 3 ? atoi(argv[3]) : 7;
  ed_params p;
  memset(&p, 0, sizeof(p));
  p.norb = norb; p.nspin = 1; p.nbath = nbath; p.hfmode = 1; p.uloc[0] = 2.0; p.uloc[1] = 2.0;
  for (int o = 0; o < norb; o++)
    for (int k = 0; k < nbath; k++) {
      p.bath_e[0][o][k] = -2.0 + 4.0 * k / (nbath - 1);
      p.bath_v[0][o][k] = 1.0 / sqrt((double)nbath);
    }
  ed_sector* s;
  if (ed_sector_create(&p, q, q, ED_STORED | ED_REAL, 0, nullptr, &s)) {
    printf("create failed: %s\n", ed_gpu_last_error());
    return 1;
  }
  ed_sell_view v;
  ed_sector_sell_view(s, &v);
  const int64_t dim = v.dim, ns = v.nslice;
  std::vector<int64_t> sp(ns + 1);
  CK(hipMemcpy(sp.data(), v.sptr, (ns + 1) * 8, hipMemcpyDeviceToHost));
  int wmin = 1 << 30, wmax = 0;
  for (int64_t i = 0; i < ns; i++) {
    int w = (int)((sp[i + 1] - sp[i]) / 64);
    wmin = w < wmin ? w : wmin;
    wmax = w > wmax ? w : wmax;
  }
  std::vector<double> hx(dim);
  for (int64_t i = 0; i < dim; i++) hx[i] = sin((double)(i + 1));
  double *x, *y, *yr;
  CK(hipMalloc(&x, dim * 8));
  CK(hipMalloc(&y, dim * 8));
  CK(hipMalloc(&yr, dim * 8));
  CK(hipMemcpy(x, hx.data(), dim * 8, hipMemcpyHostToDevice));
  ed_sector_hxv_dev_path(s, 0, 0, x, yr, nullptr);
  CK(hipDeviceSynchronize());
  std::vector<double> ref(dim), got(dim);
  CK(hipMemcpy(ref.data(), yr, dim * 8, hipMemcpyDeviceToHost));
  const double B = 12.0 * (double)(v.slots + dim) + 8.0 * (dim + 1) + 16.0 * dim;  // alg bytes (nnz incl diag; padding 0 here)
  printf("dim=%ld nslice=%ld slots=%ld width[min,max]=[%d,%d] alg_bytes=%.0f\n", (long)dim, (long)ns,
         (long)v.slots, wmin, wmax, B);
  const double* dg = (const double*)v.diag;
  const double* vl = (const double*)v.vals;
  struct Var {
    const char* name;
    kfn f;
    int bs;
    int grid;
  };
  int64_t nthr = ns * 64;
  int full256 = (int)((nthr + 255) / 256), full512 = (int)((nthr + 511) / 512);
  std::vector<Var> vars = {
      {"v0 lib (256, grid 8192)", v0<256>, 256, 8192},
      {"v0 (256, full grid)", v0<256>, 256, full256},
      {"v1 C8 (256, 8192)", v1<256, 8, 0>, 256, 8192},
      {"v1 C8 nt (256, 8192)", v1<256, 8, 1>, 256, 8192},
      {"v1 C8 (256, full)", v1<256, 8, 0>, 256, full256},
      {"v1 C8 nt (256, full)", v1<256, 8, 1>, 256, full256},
      {"v1 C4 nt (256, full)", v1<256, 4, 1>, 256, full256},
      {"v1 C16 nt (256, full)", v1<256, 16, 1>, 256, full256},
      {"v1 C8 nt (512, full)", v1<512, 8, 1>, 512, full512},
      {"v1 C8 nt (256, 2048)", v1<256, 8, 1>, 256, 2048},
  };
  if (wmin == wmax && wmin == 14) {
    vars.push_back({"v3 W14 (256, full)", v3<256, 14, 0>, 256, full256});
    vars.push_back({"v3 W14 nt (256, full)", v3<256, 14, 1>, 256, full256});
    vars.push_back({"v3 W14 nt (256, 8192)", v3<256, 14, 1>, 256, 8192});
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  for (int rep = 0; rep < 2; rep++)
    for (auto& V : vars) {
      CK(hipMemset(y, 0, dim * 8));
      for (int it = 0; it < 3; it++)
        hipLaunchKernelGGL(V.f, dim3(V.grid), dim3(V.bs), 0, 0, dg, v.sptr, v.cols, vl, x, y, dim, ns);
      CK(hipDeviceSynchronize());
      CK(hipMemcpy(got.data(), y, dim * 8, hipMemcpyDeviceToHost));
      bool ok = memcmp(got.data(), ref.data(), dim * 8) == 0;
      const int N = 30;
      CK(hipEventRecord(e0, 0));
      for (int it = 0; it < N; it++)
        hipLaunchKernelGGL(V.f, dim3(V.grid), dim3(V.bs), 0, 0, dg, v.sptr, v.cols, vl, x, y, dim, ns);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      ms /= N;
      if (rep == 1)
        printf("%-28s %8.4f ms  %7.1f GB/s  %5.1f%%  %s\n", V.name, ms, B / (ms * 1e-3) / 1e9,
               100.0 * B / (ms * 1e-3) / 8e12, ok ? "bit-exact" : "MISMATCH");
    }
  ed_sector_destroy(s);
  return 0;
}
