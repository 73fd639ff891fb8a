// stage_variants.hip — experiment tool (not part of the product): A/B timing
// of the packed stored H·v (k_spmv_pk's arithmetic) with the row's own idw
// block of v staged in LDS, on a sector built by libedgpu.so.  Every variant
// must reproduce the library's stored H·v bit for bit (same words, same
// dictionary values, same per-row summation order).
//
//   hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off -I include \
//     tools/stage_variants.hip -L dmft-ed_amd -ledgpu -Wl,-rpath,'$ORIGIN/../dmft-ed_amd' -o tools/stage_variants
//   tools/stage_variants [norb nbath q]        (default 1 13 7: the Nlevels=28 (7,7) sector)
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <map>
#include <vector>

#include "../include/ed_gpu.h"

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__); \
      exit(1);                                                                      \
    }                                                                               \
  } while (0)

constexpr int kShift = 24;
constexpr uint32_t kColMask = (1u << kShift) - 1;

// P0: k_spmv_pk's loop (one thread per row, chunks of 16, dictionary in LDS,
// XCD row ranges), non-temporal word and diagonal loads
template <int STREAM>
__global__ void __launch_bounds__(256) p0(const double* __restrict__ diag, const int64_t* __restrict__ sptr,
                                          const uint32_t* __restrict__ words, const double* __restrict__ dict,
                                          const double* __restrict__ x, double* __restrict__ y, int64_t dim,
                                          int64_t nslice) {
  __shared__ double sd[256];
  sd[threadIdx.x] = dict[threadIdx.x];
  __syncthreads();
  int64_t b = blockIdx.x;
  b = (b & 7) * (gridDim.x >> 3) + (b >> 3);
  for (int64_t i = b * 256 + threadIdx.x; i < nslice * 64; i += (int64_t)gridDim.x * 256) {
    if (i >= dim) continue;
    const int64_t s = (int64_t)__builtin_amdgcn_readfirstlane((int)(i >> 6));
    const int64_t s0 = sptr[s];
    const int w = (int)((sptr[s + 1] - s0) >> 6);
    const uint32_t* wp = words + s0 + (i & 63);
    const double xi = x[i];
    double acc = 0.0 + __builtin_nontemporal_load(diag + i) * xi;
    for (int k0 = 0; k0 < w; k0 += 16) {
      uint32_t c[16];
#pragma unroll
      for (int k = 0; k < 16; k++) c[k] = (k0 + k < w) ? __builtin_nontemporal_load(wp + 64 * (k0 + k)) : (uint32_t)i;
      double g[16], h[16];
#pragma unroll
      for (int k = 0; k < 16; k++) {
        g[k] = STREAM ? x[i] : x[c[k] & kColMask];
        h[k] = sd[c[k] >> kShift];
      }
#pragma unroll
      for (int k = 0; k < 16; k++)
        if (k0 + k < w) acc = acc + h[k] * g[k];
    }
    y[i] = acc;
  }
}

// P1: one task per workgroup = a run of slices whose rows lie (mostly) in
// one idw block; that block of x (the window) is staged in LDS and every
// entry whose column falls in the window is gathered from LDS, the others
// from global memory.  XCD-aware task order (each XCD a contiguous range).
struct Task {
  int32_t s0, s1;    // slices [s0, s1)
  int32_t wlo, wlen; // window rows
};

template <int WMAX, int BS>
__global__ void __launch_bounds__(BS) p1(const double* __restrict__ diag, const int64_t* __restrict__ sptr,
                                         const uint32_t* __restrict__ words, const double* __restrict__ dict,
                                         const double* __restrict__ x, double* __restrict__ y, int64_t dim,
                                         const Task* __restrict__ tasks, int ntask) {
  __shared__ double sd[256];
  __shared__ double xw[WMAX];
  for (int t = threadIdx.x; t < 256; t += BS) sd[t] = dict[t];
  int b = blockIdx.x;
  b = (b & 7) * (gridDim.x >> 3) + (b >> 3);
  if (b >= ntask) return;
  const Task T = tasks[b];
  for (int t = threadIdx.x; t < T.wlen; t += BS) xw[t] = x[T.wlo + t];
  __syncthreads();
  const int64_t r0 = (int64_t)T.s0 * 64, r1 = (int64_t)T.s1 * 64;
  for (int64_t i = r0 + threadIdx.x; i < r1; i += BS) {
    if (i >= dim) continue;
    const int64_t s = (int64_t)__builtin_amdgcn_readfirstlane((int)(i >> 6));
    const int64_t s0 = sptr[s];
    const int w = (int)((sptr[s + 1] - s0) >> 6);
    const uint32_t* wp = words + s0 + (i & 63);
    const uint32_t oi = (uint32_t)(i - T.wlo);
    const double xi = oi < (uint32_t)T.wlen ? xw[oi] : x[i];
    double acc = 0.0 + __builtin_nontemporal_load(diag + i) * xi;
    for (int k0 = 0; k0 < w; k0 += 16) {
      uint32_t c[16];
#pragma unroll
      for (int k = 0; k < 16; k++) c[k] = (k0 + k < w) ? __builtin_nontemporal_load(wp + 64 * (k0 + k)) : (uint32_t)i;
      double g[16], h[16];
#pragma unroll
      for (int k = 0; k < 16; k++) {
        const uint32_t col = c[k] & kColMask;
        const uint32_t o = col - (uint32_t)T.wlo;
        if (o < (uint32_t)T.wlen) g[k] = xw[o];
        else g[k] = x[col];
        h[k] = sd[c[k] >> kShift];
      }
#pragma unroll
      for (int k = 0; k < 16; k++)
        if (k0 + k < w) acc = acc + h[k] * g[k];
    }
    y[i] = acc;
  }
}

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
  const int ns = (nbath + 1) * norb;
  ed_sector* s;
  if (ed_sector_create(&p, q, q, ED_STORED | ED_REAL, 0, nullptr, &s)) {
    printf("create failed: %s\n", ed_gpu_last_error());
    return 1;
  }
  ed_sell_view v;
  ed_sector_sell_view(s, &v);
  const int64_t dim = v.dim, nsl = v.nslice;
  std::vector<int64_t> sp(nsl + 1);
  CK(hipMemcpy(sp.data(), v.sptr, (nsl + 1) * 8, hipMemcpyDeviceToHost));
  const int64_t slots = sp[nsl];
  // host packing: dictionary of the distinct value bit patterns
  std::vector<int32_t> hc(slots);
  std::vector<double> hv(slots);
  CK(hipMemcpy(hc.data(), v.cols, slots * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hv.data(), v.vals, slots * 8, hipMemcpyDeviceToHost));
  std::map<uint64_t, int> dix;
  std::vector<double> dict(256, 0.0);
  std::vector<uint32_t> hw(slots);
  for (int64_t k = 0; k < slots; k++) {
    uint64_t key;
    memcpy(&key, &hv[k], 8);
    auto it = dix.find(key);
    int id;
    if (it == dix.end()) {
      id = (int)dix.size();
      if (id >= 256) { printf("> 256 values\n"); return 1; }
      dix[key] = id;
      dict[id] = hv[k];
    } else {
      id = it->second;
    }
    hw[k] = (uint32_t)hc[k] | ((uint32_t)id << kShift);
  }
  std::vector<double>().swap(hv);
  std::vector<int32_t>().swap(hc);
  std::vector<uint32_t> map(dim);
  ed_sector_map(s, map.data());
  // blocks (idw changes) and tasks
  std::vector<int64_t> bstart;  // block of row i: largest bstart <= i
  for (int64_t i = 0; i < dim; i++)
    if (i == 0 || (map[i] >> ns) != (map[i - 1] >> ns)) bstart.push_back(i);
  bstart.push_back(dim);
  constexpr int WMAX = 3456;
  std::vector<Task> tasks;
  {
    size_t bi = 0;
    int64_t sl = 0;
    while (sl < nsl) {
      const int64_t mid = std::min<int64_t>(sl * 64 + 32, dim - 1);
      while (bstart[bi + 1] <= mid) bi++;
      const int64_t blo = bstart[bi], bhi = bstart[bi + 1];
      int64_t se = sl + 1;
      while (se < nsl && std::min<int64_t>(se * 64 + 32, dim - 1) < bhi) se++;
      Task t;
      t.s0 = (int32_t)sl;
      t.s1 = (int32_t)se;
      t.wlo = (int32_t)blo;
      t.wlen = (int32_t)std::min<int64_t>(bhi - blo, WMAX);
      tasks.push_back(t);
      sl = se;
    }
  }
  const int ntask = (int)tasks.size();
  const int gtask = (ntask + 7) / 8 * 8;
  printf("dim=%ld nslice=%ld slots=%ld ndict=%d blocks=%zu tasks=%d\n", (long)dim, (long)nsl, (long)slots,
         (int)dix.size(), bstart.size() - 1, ntask);
  uint32_t* dw;
  double *dd, *x, *y, *yr;
  Task* dt;
  CK(hipMalloc(&dw, slots * 4));
  CK(hipMalloc(&dd, 256 * 8));
  CK(hipMalloc(&dt, ntask * sizeof(Task)));
  CK(hipMemcpy(dw, hw.data(), slots * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dd, dict.data(), 256 * 8, hipMemcpyHostToDevice));
  CK(hipMemcpy(dt, tasks.data(), ntask * sizeof(Task), hipMemcpyHostToDevice));
  std::vector<double> hx(dim);
  for (int64_t i = 0; i < dim; i++) hx[i] = sin((double)(i + 1));
  CK(hipMalloc(&x, dim * 8));
  CK(hipMalloc(&y, dim * 8));
  CK(hipMalloc(&yr, dim * 8));
  CK(hipMemcpy(x, hx.data(), dim * 8, hipMemcpyHostToDevice));
  ed_sector_hxv_dev_path(s, 0, 0, x, yr, nullptr);
  CK(hipDeviceSynchronize());
  std::vector<double> ref(dim), got(dim);
  CK(hipMemcpy(ref.data(), yr, dim * 8, hipMemcpyDeviceToHost));
  const double B = 4.0 * slots + 8.0 * (nsl + 1) + 24.0 * dim;  // own bytes of the packed kernel
  const double* dg = (const double*)v.diag;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int g0 = (int)std::min<int64_t>((nsl * 64 + 255) / 256, 65536) & ~7;
  auto run = [&](const char* name, auto launch, bool check) {
    CK(hipMemset(y, 0, dim * 8));
    for (int it = 0; it < 3; it++) launch();
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(got.data(), y, dim * 8, hipMemcpyDeviceToHost));
    const bool ok = memcmp(got.data(), ref.data(), dim * 8) == 0;
    const int N = 30;
    CK(hipEventRecord(e0, 0));
    for (int it = 0; it < N; it++) launch();
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= N;
    printf("%-34s %8.4f ms  own %7.1f GB/s  frac %.3f  %s\n", name, ms, B / (ms * 1e-3) / 1e9,
           B / (ms * 1e-3) / 8e12, check ? (ok ? "bit-exact" : "MISMATCH") : "(timing only)");
  };
  for (int rep = 0; rep < 2; rep++) {
    run("p0 packed (k_spmv_pk form)", [&] {
      hipLaunchKernelGGL(p0<0>, dim3(g0), dim3(256), 0, 0, dg, v.sptr, dw, dd, x, y, dim, nsl);
    }, true);
    run("p0 stream floor (gathers own row)", [&] {
      hipLaunchKernelGGL(p0<1>, dim3(g0), dim3(256), 0, 0, dg, v.sptr, dw, dd, x, y, dim, nsl);
    }, false);
    run("p1 staged block 256", [&] {
      hipLaunchKernelGGL((p1<WMAX, 256>), dim3(gtask), dim3(256), 0, 0, dg, v.sptr, dw, dd, x, y, dim, dt, ntask);
    }, true);
    run("p1 staged block 512", [&] {
      hipLaunchKernelGGL((p1<WMAX, 512>), dim3(gtask), dim3(512), 0, 0, dg, v.sptr, dw, dd, x, y, dim, dt, ntask);
    }, true);
    run("p1 staged block 1024", [&] {
      hipLaunchKernelGGL((p1<WMAX, 1024>), dim3(gtask), dim3(1024), 0, 0, dg, v.sptr, dw, dd, x, y, dim, dt, ntask);
    }, true);
  }
  ed_sector_destroy(s);
  return 0;
}
