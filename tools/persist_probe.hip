// persist_probe.hip — A/B timing of one-workgroup persistent Lanczos layouts
// on the configs[1] (Norb=1 Nbath=7, (4,4)) sector structure (experiment
// tool, not part of the product; synthetic values of the same sparsity).
//
//   V0  ELL words {col | dictionary offset} in registers, dictionary + v +
//       diagonal in LDS (the library's MODE 2)
//   V1  V0 without the dictionary read (timing only: wrong values)
//   V2  V0 with conflict-free gathers (timing only)
//   V3  no off-diagonal work (barriers + reductions + epilogue floor)
//   V4  Kronecker register layout: thread (g, iu) owns rows (g + G*r, iu);
//       the up-hop entries (col, value) are the same for all its rows and sit
//       in registers once; the down-hop entries (col, value) per row in
//       registers; no dictionary; diagonal in LDS
//   V5  V4 with the diagonal in registers
//
// build: hipcc -O3 --offload-arch=gfx950 -std=c++17 -ffp-contract=off \
//          -I dmft-ed_amd/csrc tools/persist_probe.hip -o tools/persist_probe
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <map>
#include <vector>

#include "ed_persist.hpp"

using namespace edg;

#define CK(x)                                                                            \
  do {                                                                                   \
    hipError_t e = (x);                                                                  \
    if (e != hipSuccess) {                                                               \
      printf("HIP error %s at %s:%d\n", hipGetErrorString(e), __FILE__, __LINE__);       \
      exit(1);                                                                           \
    }                                                                                    \
  } while (0)

constexpr int NS = 8, NE = 4;      // sites per spin, electrons per spin
constexpr int NT = 512;
constexpr int W = 8, DEG = 4;      // entries per row, up (= down) hops per row

struct Args {
  const uint32_t* pk;   // V0: [RPT*W][NT]
  const double* dict;
  int ndict;
  const double* diag;   // [dim]
  // V4/V5
  const int* upc;       // [DEG][du] target up rank
  const double* upv;    // [DEG][du]
  const int* dwc;       // [DEG][dd]
  const double* dwv;    // [DEG][dd]
  int du, dd, G;
  double* R;
  double* alpha;
  double* beta;
  int dim, niter;
};

template <int NT, bool DPP, bool TAIL = true>
__device__ __forceinline__ double bsum(double v, double* ws) {
  if constexpr (!DPP) return pblock_sum<NT, TAIL>(v, ws);
  v = wave_sum_dpp(v);
  if ((threadIdx.x & 63) == 63) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) t = t + ws[w];
  if constexpr (TAIL) __syncthreads();
  return t;
}

constexpr int O_PAD = 1, O_DPP = 2, O_XREG = 4;

template <int V, int RPT, int OPT = 0>
__global__ void __launch_bounds__(NT) k_probe(Args a) {
  extern __shared__ __align__(16) unsigned char smem[];
  __shared__ double ws[NT / 64];
  __shared__ double ws2[NT / 64];
  constexpr bool PAD = OPT & O_PAD, DPP = OPT & O_DPP, XREG = OPT & O_XREG;
  const int tid = threadIdx.x;
  const int dim = a.dim;
  const int vdim = PAD ? NT * RPT : dim;  // LDS rows (pad rows stay 0)
  const int dbytes = ((a.ndict * 8 + 15) & ~15);
  double* vl = (double*)(smem + dbytes);
  double* dg = (double*)(smem + dbytes + ((vdim * 8 + 15) & ~15));
  for (int t = tid; t < a.ndict; t += NT) ((double*)smem)[t] = a.dict[t];
  for (int t = tid; t < vdim; t += NT) dg[t] = t < dim ? a.diag[t] : 0.0;
  constexpr bool KR = V >= 4;
  // row of slot r: row0 + r * stride while r < nr (PAD: every slot, pad rows >= dim)
  const int du = a.du;
  const int g = tid / du, iu = tid - g * du;
  const bool act = !KR || g < a.G;
  const int row0 = KR ? g * du + iu : tid;
  const int stride = KR ? a.G * du : NT;
  const int nr = !act ? 0 : KR ? (a.dd - g + a.G - 1) / a.G : (dim - tid + NT - 1) / NT;
#define ROW(r) (row0 + (r) * stride)
#define OK(r) (PAD || (r) < nr)
#define VALID(r) ((r) < nr)
  uint32_t pk[KR ? 1 : RPT * W];
  int ucol[KR ? DEG : 1];
  double uval[KR ? DEG : 1];
  int dcol[KR ? RPT * DEG : 1];
  double dval[KR ? RPT * DEG : 1];
  double dgr[V == 5 ? RPT : 1];
  if constexpr (!KR) {
#pragma unroll
    for (int k = 0; k < RPT * W; k++) pk[k] = a.pk[k * NT + tid];
  } else {
#pragma unroll
    for (int e = 0; e < DEG; e++) {
      ucol[e] = act ? a.upc[e * du + iu] * 8 : 0;
      uval[e] = act ? a.upv[e * du + iu] : 0.0;
    }
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      const int iw = g + a.G * r;
#pragma unroll
      for (int e = 0; e < DEG; e++) {
        const bool ok = VALID(r);
        dcol[r * DEG + e] = ok ? (a.dwc[e * a.dd + iw] * du + iu) * 8 : 0;
        dval[r * DEG + e] = ok ? a.dwv[e * a.dd + iw] : 0.0;
      }
      if constexpr (V == 5) dgr[r] = VALID(r) ? a.diag[ROW(r)] : 0.0;
    }
  }
  double p[RPT];
  double nrm = 0.0;
#pragma unroll
  for (int r = 0; r < RPT; r++) {
    p[r] = 0.0;
    if (OK(r)) {
      const double x = VALID(r) ? a.R[ROW(r)] : 0.0;
      vl[ROW(r)] = x;
      nrm += x * x;
    }
  }
  const double n2 = pblock_sum<NT>(nrm, ws);
  const double inv0 = 1.0 / sqrt(n2);
#pragma unroll
  for (int r = 0; r < RPT; r++)
    if (OK(r)) vl[ROW(r)] *= inv0;
  __syncthreads();
  double b = 0.0;
  const unsigned char* dct = smem;
  for (int it = 0; it < a.niter; it++) {
    if constexpr (!KR) {
#pragma unroll
      for (int e = 0; e < RPT * W; e++) asm volatile("" : "+v"(pk[e]));
    } else {
#pragma unroll
      for (int e = 0; e < RPT * DEG; e++) asm volatile("" : "+v"(dcol[e]));
    }
    double w[RPT], xs[XREG ? RPT : 1];
    double ap = 0.0;
#pragma unroll
    for (int r = 0; r < RPT; r++) {
      w[r] = 0.0;
      const int i = ROW(r);
      if (OK(r)) {
        const double xi = vl[i];
        if constexpr (XREG) xs[r] = xi;
        double acc;
        if constexpr (V == 5) acc = dgr[r] * xi;
        else acc = dg[i] * xi;
        if constexpr (V <= 2) {
#pragma unroll
          for (int e = 0; e < W; e++) {
            const uint32_t x = pk[r * W + e];
            double h;
            if constexpr (V == 1) h = 0.25;
            else h = *(const double*)(dct + ((x >> kPkColBits) & kPkOffMask));
            const double xv = V == 2 ? vl[(i + 64 * e) % dim] : vl[x & kPkColMask];
            acc = fmac(acc, h, xv);
          }
        } else if constexpr (KR) {
          const unsigned char* rb = (const unsigned char*)(vl + (i - iu));  // row iw of V
#pragma unroll
          for (int e = 0; e < DEG; e++) acc = fmac(acc, uval[e], *(const double*)(rb + ucol[e]));
#pragma unroll
          for (int e = 0; e < DEG; e++)
            acc = fmac(acc, dval[r * DEG + e], *(const double*)((const unsigned char*)vl + dcol[r * DEG + e]));
        }
        w[r] = acc - b * p[r];
        ap += xi * w[r];
      }
    }
    const double alpha = bsum<NT, DPP, false>(ap, ws);
    double bp = 0.0;
#pragma unroll
    for (int r = 0; r < RPT; r++)
      if (OK(r)) {
        const double xi = XREG ? xs[r] : vl[ROW(r)];
        w[r] = w[r] - alpha * xi;
        bp += w[r] * w[r];
      }
    const double bn = sqrt(bsum<NT, DPP, false>(bp, ws2));
    if (tid == 0) {
      a.alpha[it] = alpha;
      a.beta[it + 1] = bn;
    }
    const double inv = 1.0 / bn;
#pragma unroll
    for (int r = 0; r < RPT; r++)
      if (OK(r)) {
        p[r] = XREG ? xs[r] : vl[ROW(r)];
        vl[ROW(r)] = inv * w[r];
      }
    b = bn;
    __syncthreads();
  }
}

static int popc(int x) { return __builtin_popcount(x); }

int main(int argc, char** argv) {
  const int niter = argc > 1 ? atoi(argv[1]) : 512;
  // basis of one spin: patterns with NE of NS bits, ascending (rank order)
  std::vector<int> pat, rank(1 << NS, -1);
  for (int x = 0; x < (1 << NS); x++)
    if (popc(x) == NE) { rank[x] = (int)pat.size(); pat.push_back(x); }
  const int du = (int)pat.size(), dd = du, dim = du * dd;
  srand(12345);
  auto rnd = [] { return (double)rand() / RAND_MAX; };
  double Vk[NS], eps[NS];
  for (int k = 0; k < NS; k++) { Vk[k] = 0.1 + 0.9 * rnd(); eps[k] = -2 + 4 * rnd(); }
  // hop table: imp (site 0) <-> bath k, in k order
  std::vector<int> hc(DEG * du);
  std::vector<double> hv(DEG * du);
  for (int u = 0; u < du; u++) {
    int e = 0;
    for (int k = 1; k < NS; k++) {
      const int x = pat[u];
      if (((x >> 0) & 1) == ((x >> k) & 1)) continue;
      const int y = x ^ 1 ^ (1 << k);
      const int sg = (popc(x & ((1 << k) - 2)) & 1) ? -1 : 1;
      hc[e * du + u] = rank[y];
      hv[e * du + u] = sg * Vk[k];
      e++;
    }
    if (e != DEG) { printf("bad degree %d\n", e); return 1; }
  }
  std::vector<double> diag(dim);
  for (int i = 0; i < dim; i++) {
    const int iw = i / du, iu = i % du;
    double d = 0;
    for (int k = 0; k < NS; k++) d += eps[k] * (((pat[iu] >> k) & 1) + ((pat[iw] >> k) & 1));
    d += 2.0 * (pat[iu] & 1) * (pat[iw] & 1);
    diag[i] = d;
  }
  // V0 packed words: row i entries = up hops then down hops
  constexpr int RPT0 = 10;
  std::map<double, int> dix;
  std::vector<double> dict{0.0};
  dix[0.0] = 0;
  auto did = [&](double v) {
    auto it = dix.find(v);
    if (it != dix.end()) return it->second;
    int id = (int)dict.size();
    dict.push_back(v);
    dix[v] = id;
    return id;
  };
  std::vector<uint32_t> pk((size_t)RPT0 * W * NT, 0);
  for (int r = 0; r < RPT0; r++)
    for (int t = 0; t < NT; t++) {
      const int i = t + NT * r;
      for (int e = 0; e < W; e++) {
        uint32_t wd = 0;
        if (i < dim) {
          const int iw = i / du, iu = i % du;
          int col;
          double v;
          if (e < DEG) { col = iw * du + hc[e * du + iu]; v = hv[e * du + iu]; }
          else { col = hc[(e - DEG) * du + iw] * du + iu; v = hv[(e - DEG) * du + iw]; }
          wd = (uint32_t)col | ((uint32_t)(did(v) * 8) << kPkColBits);
        }
        pk[((size_t)r * W + e) * NT + t] = wd;
      }
    }
  printf("dim %d du %d ndict %zu\n", dim, du, dict.size());
  std::vector<double> x0(dim);
  for (int i = 0; i < dim; i++) x0[i] = sin(i + 1.0);

  auto up = [](const void* h, size_t n) {
    void* d;
    CK(hipMalloc(&d, n));
    CK(hipMemcpy(d, h, n, hipMemcpyHostToDevice));
    return d;
  };
  Args a{};
  a.pk = (uint32_t*)up(pk.data(), pk.size() * 4);
  a.dict = (double*)up(dict.data(), dict.size() * 8);
  a.ndict = (int)dict.size();
  a.diag = (double*)up(diag.data(), dim * 8);
  a.upc = (int*)up(hc.data(), hc.size() * 4);
  a.upv = (double*)up(hv.data(), hv.size() * 8);
  a.dwc = a.upc;
  a.dwv = a.upv;
  a.du = du;
  a.dd = dd;
  a.G = NT / du;
  a.R = (double*)up(x0.data(), dim * 8);
  a.dim = dim;
  a.niter = niter;
  CK(hipMalloc(&a.alpha, (niter + 2) * 8));
  CK(hipMalloc(&a.beta, (niter + 2) * 8));
  const size_t lds = ((dict.size() * 8 + 15) & ~15) + ((NT * 10 * 8 + 15) & ~15) * 2;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> alpha_ref;
  auto run = [&](auto fn, const char* name) {
    CK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    float best = 1e30f;
    for (int rep = 0; rep < 6; rep++) {
      CK(hipEventRecord(e0));
      hipLaunchKernelGGL(fn, dim3(1), dim3(NT), lds, 0, a);
      CK(hipEventRecord(e1));
      CK(hipEventSynchronize(e1));
      float ms;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (rep) best = std::min(best, ms);
    }
    std::vector<double> al(niter);
    CK(hipMemcpy(al.data(), a.alpha, niter * 8, hipMemcpyDeviceToHost));
    if (alpha_ref.empty()) alpha_ref = al;
    double err = 0;
    for (int k = 0; k < 20; k++) err = std::max(err, fabs(al[k] - alpha_ref[k]));
    printf("%-4s %8.3f us/step  alpha[0..19] max |d| vs V0 %.2e\n", name, 1e3 * best / niter, err);
  };
  const int RPTK = (dd + a.G - 1) / a.G;
  printf("G %d RPT(kron) %d\n", a.G, RPTK);
  run(k_probe<0, RPT0>, "V0");
  run(k_probe<1, RPT0>, "V1");
  run(k_probe<2, RPT0>, "V2");
  run(k_probe<3, RPT0>, "V3");
  if (RPTK == 10) {
    run(k_probe<4, 10>, "V4");
    run(k_probe<5, 10>, "V5");
  }
  run(k_probe<0, RPT0, O_PAD>, "V0p");
  run(k_probe<0, RPT0, O_DPP>, "V0d");
  run(k_probe<0, RPT0, O_XREG>, "V0x");
  run(k_probe<0, RPT0, O_PAD | O_DPP | O_XREG>, "V0a");
  run(k_probe<3, RPT0, O_PAD | O_DPP | O_XREG>, "V3a");
  if (RPTK == 10) {
    run(k_probe<4, 10, O_PAD | O_DPP | O_XREG>, "V4a");
    run(k_probe<5, 10, O_PAD | O_DPP | O_XREG>, "V5a");
  }
  return 0;
}
