// ed_trlan.hpp — kernels of the device thick-restart Lanczos (ARPACK path).
//
// The reference's default spectrum solver is ARPACK through SciFortran's
// sp_eigh (ED_DIAG.f90:145-167: Neigen=min(dim,6), ncv=Nblock=23,
// which="SR", tol=lanc_tolerance).  Here the Krylov basis V (dim x ncv,
// column-major, column c at V + c*dim) stays in HBM and every O(dim) step is
// a kernel; only the ncv x ncv projected matrix goes to the host.
//   k_vdot_part   partial h_c = <V_c, w> for a block of columns (CGS2 pass)
//   k_vdot_fin    sum of the per-block partials -> h (device)
//   k_vaxpy       w -= sum_c V_c h_c
//   k_rotate      X_k = sum_c V_c Y(c,k)      (restart / Ritz vectors)
//   k_scale_into  V_{j+1} = w / beta
//   k_cgs         fused CGS2 sweep: x -= V h (optional), then the block
//                 partials of <V_c, x> and/or |x|^2 from the same V loads, so
//                 a CGS2 orthogonalisation streams V three times, not four
// All loops are grid-strided over rows with coalesced column accesses.
#pragma once
#include "ed_kernels.hpp"
#include "ed_persist.hpp"

namespace edg {

constexpr int kVCols = 8;  // columns handled per pass of k_vdot_part

// conj(a) * b
__device__ __forceinline__ double2 cdotc(double2 a, double2 b) {
  return make_double2(a.x * b.x + a.y * b.y, a.x * b.y - a.y * b.x);
}
__device__ __forceinline__ double2 cdotc(double a, double b) { return make_double2(a * b, 0.0); }

// part[c * G + blockIdx.x] (re, im) = partial <V_c, w>; blockIdx.y picks the
// column chunk [8y, 8y+8) ∩ [0, ncol).
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_vdot_part(const val_t<VC>* __restrict__ V, int ncol,
                                                      const val_t<VC>* __restrict__ w, int64_t dim,
                                                      double2* __restrict__ part) {
  const int c0 = blockIdx.y * kVCols;
  double2 acc[kVCols];
#pragma unroll
  for (int c = 0; c < kVCols; c++) acc[c] = make_double2(0.0, 0.0);
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim; i += (int64_t)gridDim.x * kBlock) {
    const auto wi = w[i];
#pragma unroll
    for (int c = 0; c < kVCols; c++)
      if (c0 + c < ncol) {
        const double2 t = cdotc(V[(int64_t)(c0 + c) * dim + i], wi);
        acc[c].x += t.x;
        acc[c].y += t.y;
      }
  }
#pragma unroll
  for (int c = 0; c < kVCols; c++) {
    if (c0 + c >= ncol) break;  // uniform
    double re = block_sum(acc[c].x);
    double im = block_sum(acc[c].y);
    if (threadIdx.x == 0) part[(int64_t)(c0 + c) * gridDim.x + blockIdx.x] = make_double2(re, im);
  }
}

// h[c] = sum_b part[c*G + b] (imaginary part dropped for real vectors); one
// block per column.  coef[c] = h[c] (add == 0) or coef[c] += h[c] (add == 1).
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_vdot_fin(const double2* __restrict__ part, int G,
                                                     double2* __restrict__ h, double2* __restrict__ coef,
                                                     int add) {
  const int c = blockIdx.x;
  double re = 0.0, im = 0.0;
  for (int b = threadIdx.x; b < G; b += kBlock) {
    re += part[(int64_t)c * G + b].x;
    im += part[(int64_t)c * G + b].y;
  }
  re = block_sum(re);
  im = VC ? block_sum(im) : 0.0;
  if (threadIdx.x == 0) {
    h[c] = make_double2(re, im);
    if (add) coef[c] = make_double2(coef[c].x + re, coef[c].y + im);
    else coef[c] = make_double2(re, im);
  }
}

// w -= sum_{c<ncol} V_c h_c; with npart != nullptr also the block partials of |w|^2
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_vaxpy(const val_t<VC>* __restrict__ V, int ncol,
                                                  const double2* __restrict__ h, val_t<VC>* __restrict__ w,
                                                  int64_t dim, double* __restrict__ npart) {
  __shared__ double2 hs[64];
  for (int c = threadIdx.x; c < ncol; c += kBlock) hs[c] = h[c];
  __syncthreads();
  double n2 = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim; i += (int64_t)gridDim.x * kBlock) {
    auto x = w[i];
    for (int c = 0; c < ncol; c++) {
      const auto v = V[(int64_t)c * dim + i];
      if constexpr (VC) {
        x.x -= v.x * hs[c].x - v.y * hs[c].y;
        x.y -= v.x * hs[c].y + v.y * hs[c].x;
      } else {
        x -= v * hs[c].x;  // real vectors: coefficients are real
      }
    }
    w[i] = x;
    n2 += redot(x, x);
  }
  if (npart) {
    n2 = block_sum(n2);
    if (threadIdx.x == 0) npart[blockIdx.x] = n2;
  }
}

// beta[j] = ||w|| from the partials; alpha[j] = Re coef[j]
__global__ void __launch_bounds__(kBlock) k_trl_coef(const double* __restrict__ npart, int G,
                                                     const double2* __restrict__ coef, int j,
                                                     double* __restrict__ alpha, double* __restrict__ beta) {
  double t = 0.0;
  for (int b = threadIdx.x; b < G; b += kBlock) t += npart[b];
  t = block_sum(t);
  if (threadIdx.x == 0) {
    beta[j] = sqrt(t);
    if (alpha) alpha[j] = coef[j].x;
  }
}

// X_k = sum_{c<ncol} V_c Y[c + k*ldy] for k < nout (Y real, column-major).
// Outputs in register chunks of kVCols so V is streamed ceil(nout/8) times.
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_rotate(const val_t<VC>* __restrict__ V, int ncol,
                                                   const double* __restrict__ Y, int ldy, int nout,
                                                   val_t<VC>* __restrict__ X, int64_t dim) {
  extern __shared__ double ys[];  // ncol * nout (<= 64 * 64)
  for (int t = threadIdx.x; t < ncol * nout; t += kBlock) ys[t] = Y[(t % ncol) + (int64_t)(t / ncol) * ldy];
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim; i += (int64_t)gridDim.x * kBlock) {
    for (int k0 = 0; k0 < nout; k0 += kVCols) {
      val_t<VC> acc[kVCols];
#pragma unroll
      for (int k = 0; k < kVCols; k++) acc[k] = vzero<val_t<VC>>();
      for (int c = 0; c < ncol; c++) {
        const auto v = V[(int64_t)c * dim + i];
#pragma unroll
        for (int k = 0; k < kVCols; k++)
          if (k0 + k < nout) acc[k] = add(acc[k], scl(ys[c + (k0 + k) * ncol], v));
      }
#pragma unroll
      for (int k = 0; k < kVCols; k++)
        if (k0 + k < nout) X[(int64_t)(k0 + k) * dim + i] = acc[k];
    }
  }
}

// y = x * (1/nrm) with nrm read from device (0 -> zeros)
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_scale_into(const val_t<VC>* __restrict__ x,
                                                       val_t<VC>* __restrict__ y, const double* nrm,
                                                       int64_t dim) {
  const double inv = nrm[0] > 0.0 ? 1.0 / nrm[0] : 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim; i += (int64_t)gridDim.x * kBlock)
    y[i] = scl(inv, x[i]);
}

// k_trl_coef + k_scale_into in one launch (grid-strided): every block forms
// the same fixed-order sum of the norm partials; block 0 stores alpha/beta,
// all blocks write out = x / ||x|| (zeros for a zero norm).
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_coef_scale(const double* __restrict__ npart, int G,
                                                       const double2* __restrict__ coef, int j,
                                                       double* __restrict__ alpha, double* __restrict__ beta,
                                                       const val_t<VC>* __restrict__ x,
                                                       val_t<VC>* __restrict__ out, int64_t dim) {
  double t = 0.0;
  for (int b = threadIdx.x; b < G; b += kBlock) t += npart[b];
  t = block_sum(t);
  const double nrm = sqrt(t);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    beta[j] = nrm;
    if (alpha) alpha[j] = coef[j].x;
  }
  const double inv = nrm > 0.0 ? 1.0 / nrm : 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim; i += (int64_t)gridDim.x * kBlock)
    out[i] = scl(inv, x[i]);
}

// Fused CGS sweep over the rows of x (one column group of up to NC columns
// held in registers per row):
//   hin != nullptr : x_i -= sum_{c<ncol} V_c,i hin_c   (written back)
//   part != nullptr: part[c*G + b] = block partial of <V_c, x> after the update
//   npart != nullptr: npart[b]     = block partial of |x|^2 after the update
// The row loop, the per-thread accumulation order and the subtraction order
// are those of k_vdot_part / k_vaxpy; the block sums use DPP wave sums and one
// barrier for all 2*NC+1 partials.
template <bool VC, int NC>
__global__ void __launch_bounds__(kBlock) k_cgs(const val_t<VC>* __restrict__ V, int ncol,
                                                const double2* __restrict__ hin,
                                                val_t<VC>* __restrict__ x, int64_t dim,
                                                double2* __restrict__ part, double* __restrict__ npart,
                                                const double2* __restrict__ pin = nullptr, int gin = 0,
                                                double2* __restrict__ coef = nullptr, int add = 0) {
  constexpr int NW = kBlock / 64;
  constexpr int NR = (VC ? 2 * NC : NC) + 1;  // partial slots per wave
  __shared__ double2 hs[NC];
  __shared__ double red[NW][NR];
  if (pin) {
    // the previous pass's coefficients from its block partials (k_vdot_fin
    // folded in: small sectors, gin x ncol partials): every block forms the
    // same sums in the same order (wave c mod NW, lanes strided, DPP sum);
    // block 0 also records them (coef = h, or coef += h)
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    for (int c = wv; c < ncol; c += NW) {  // wave-uniform
      double re = 0.0, im = 0.0;
      for (int b = lane; b < gin; b += 64) {
        re += pin[(int64_t)c * gin + b].x;
        if constexpr (VC) im += pin[(int64_t)c * gin + b].y;
      }
      re = wave_sum_dpp(re);
      if constexpr (VC) im = wave_sum_dpp(im);
      if (lane == 63) {
        hs[c] = make_double2(re, im);
        if (coef && blockIdx.x == 0) coef[c] = add ? make_double2(coef[c].x + re, coef[c].y + im) : make_double2(re, im);
      }
    }
    __syncthreads();
  } else if (hin) {
    for (int c = threadIdx.x; c < ncol; c += kBlock) hs[c] = hin[c];
    __syncthreads();
  }
  const bool upd = hin || pin;
  double are[NC], aim[VC ? NC : 1];
#pragma unroll
  for (int c = 0; c < NC; c++) {
    are[c] = 0.0;
    if constexpr (VC) aim[c] = 0.0;
  }
  double n2 = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim; i += (int64_t)gridDim.x * kBlock) {
    val_t<VC> v[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) v[c] = c < ncol ? V[(int64_t)c * dim + i] : vzero<val_t<VC>>();
    auto xi = x[i];
    if (upd) {
#pragma unroll
      for (int c = 0; c < NC; c++) {
        if (c >= ncol) continue;  // uniform
        if constexpr (VC) {
          xi.x -= v[c].x * hs[c].x - v[c].y * hs[c].y;
          xi.y -= v[c].x * hs[c].y + v[c].y * hs[c].x;
        } else {
          xi -= v[c] * hs[c].x;
        }
      }
      x[i] = xi;
    }
    if (part) {
#pragma unroll
      for (int c = 0; c < NC; c++) {
        const double2 t = cdotc(v[c], xi);
        are[c] += t.x;
        if constexpr (VC) aim[c] += t.y;
      }
    }
    if (npart) n2 += redot(xi, xi);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (part) {
#pragma unroll
    for (int c = 0; c < NC; c++) {
      if (c >= ncol) continue;  // uniform
      const double r = wave_sum_dpp(are[c]);
      if (lane == 63) red[wv][c] = r;
      if constexpr (VC) {
        const double q = wave_sum_dpp(aim[c]);
        if (lane == 63) red[wv][NC + c] = q;
      }
    }
  }
  if (npart) {
    const double r = wave_sum_dpp(n2);
    if (lane == 63) red[wv][NR - 1] = r;
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (part && t < ncol) {
    double re = 0.0, im = 0.0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
      re = re + red[w][t];
      if constexpr (VC) im = im + red[w][NC + t];
    }
    part[(int64_t)t * gridDim.x + blockIdx.x] = make_double2(re, im);
  }
  if (npart && t == kBlock - 1) {
    double r = 0.0;
#pragma unroll
    for (int w = 0; w < NW; w++) r = r + red[w][NR - 1];
    npart[blockIdx.x] = r;
  }
}

}  // namespace edg
