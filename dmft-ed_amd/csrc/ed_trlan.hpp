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
//                 a CGS2 orthogonalisation streams V three times, not four;
//                 the second pass is conditional (ARPACK's DGKS test,
//                 dgks_skip): V streamed twice when the first pass suffices
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

// ARPACK dsaitr's DGKS test (the published algorithm of ARPACK, the
// SciFortran dependency behind sp_eigh, ED_DIAG.f90:145-167): after the first
// classical Gram-Schmidt pass w' = w - V V^H w, a second pass is made only if
// ||w'|| <= 0.717 ||w||.  From the per-block partials of |w|^2 (nA) and
// |w'|^2 (nB), summed in a fixed order by wave 0: every block of a launch
// takes the same decision.  Needs blockDim >= 64.
constexpr double kDgks2 = 0.717 * 0.717;
__device__ __forceinline__ bool dgks_skip(const double* __restrict__ nA, const double* __restrict__ nB, int G) {
  __shared__ int sk;
  if (threadIdx.x < 64) {
    double a = 0.0, b = 0.0;
    for (int i = threadIdx.x; i < G; i += 64) {
      a += nA[i];
      b += nB[i];
    }
    a = wave_sum_dpp(a);
    b = wave_sum_dpp(b);
    if (threadIdx.x == 63) sk = b > kDgks2 * a;
  }
  __syncthreads();
  return sk != 0;
}

// Local-only update.  After the shifted three-term step (EpiTrlLoc) the
// first Gram-Schmidt pass finds w nearly orthogonal to every basis column
// but the last two: the coefficients h_c, c < j-1, are rounding noise
// (round-4 measurement on configs[3] sectors: 2-30 eps of |w| at the 90th
// percentile, tools in DESIGN.md).  Subtracting V h over all j+1 columns
// then streams V a second time to correct at noise level.  When every far
// |h_c| <= 64 eps of |w - h_j v_j - h_{j-1} v_{j-1}| (= sqrt(|w|^2 -
// |h_j|^2 - |h_{j-1}|^2)), the update and the DGKS second pass act on the
// last two columns only (the second pass still taken when the norm
// dropped below 0.717 |w|); the measured far coefficients keep the decision
// honest (the dots are always taken, so a basis that drifts gets the full
// update).
constexpr double kCgsLocTol = 64.0 * 2.220446049250313e-16;
__device__ __forceinline__ double wave_max_f64(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
// Block-uniform decision from the first pass's coefficients h[0, ncol) and
// its |w|^2 partials nA[0, G) (every block sums them in the same order).
// Needs blockDim >= 64.
__device__ __forceinline__ bool cgs_loc_only(const double2* __restrict__ h, int ncol,
                                             const double* __restrict__ nA, int G) {
  __shared__ int lo;
  if (threadIdx.x < 64) {
    const int lane = threadIdx.x;
    double a = 0.0, hl = 0.0, far = 0.0;
    for (int i = lane; i < G; i += 64) a += nA[i];
    for (int c = lane; c < ncol; c += 64) {
      const double v = h[c].x * h[c].x + h[c].y * h[c].y;
      if (c >= ncol - 2) hl += v;
      else far = fmax(far, v);
    }
    a = wave_sum_dpp(a);
    hl = wave_sum_dpp(hl);
    far = wave_max_f64(far);
    if (lane == 63) {
      const double wl = a - hl;
      lo = (wl > 0.0) && (far <= kCgsLocTol * kCgsLocTol * wl);
    }
  }
  __syncthreads();
  return lo != 0;
}

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
                                                     int add, const double* dgA = nullptr,
                                                     const double* dgB = nullptr) {
  // (a local-only step folds stale partials for its far columns: unused)
  if (dgA && dgks_skip(dgA, dgB, G)) return;  // conditional second pass not needed
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
// (jc: the basis column of v_j when it differs from the alpha/beta slot j —
// the rolling two-column window of probe_screen)
static __global__ void __launch_bounds__(kBlock) k_trl_coef(const double* __restrict__ npart, int G,
                                                     const double2* __restrict__ coef, int j,
                                                     double* __restrict__ alpha, double* __restrict__ beta,
                                                     int shifted = 0, int jc = -1) {
  double t = 0.0;
  for (int b = threadIdx.x; b < G; b += kBlock) t += npart[b];
  t = block_sum(t);
  if (threadIdx.x == 0) {
    beta[j] = sqrt(t);
    const int c = jc >= 0 ? jc : j;
    if (alpha) alpha[j] = shifted ? alpha[j - 1] + coef[c].x : coef[c].x;  // (EpiTrlLoc)
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

// In place: V_k = sum_{c<ncol} V_c Y[c + k*ldy] for k < nout <= ncol <= NCM.
// Each thread holds its row's ncol basis entries in registers before any
// output is stored, so the rotation overwrites the basis columns directly
// (no rotation buffer + copy back: 2·nout·dim elements less per restart);
// same products and summation order as k_rotate.
template <bool VC, int NCM>
__global__ void __launch_bounds__(kBlock) k_rotate_ip(val_t<VC>* __restrict__ V, int ncol,
                                                      const double* __restrict__ Y, int ldy, int nout,
                                                      int64_t dim) {
  __shared__ double ys[NCM * NCM];
  for (int t = threadIdx.x; t < ncol * nout; t += kBlock) ys[t] = Y[(t % ncol) + (int64_t)(t / ncol) * ldy];
  __syncthreads();
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim; i += (int64_t)gridDim.x * kBlock) {
    val_t<VC> v[NCM];
#pragma unroll
    for (int c = 0; c < NCM; c++) v[c] = c < ncol ? V[(int64_t)c * dim + i] : vzero<val_t<VC>>();
    for (int k = 0; k < nout; k++) {
      val_t<VC> acc = vzero<val_t<VC>>();
#pragma unroll
      for (int c = 0; c < NCM; c++)
        if (c < ncol) acc = add(acc, scl(ys[c + k * ncol], v[c]));
      V[(int64_t)k * dim + i] = acc;
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

// w += a * x on the raw doubles (complex vectors as interleaved pairs): the
// degeneracy screen's start vector, a hash vector plus the next Ritz vector
__global__ void __launch_bounds__(kBlock) k_mix_hint(double* __restrict__ w, const double* __restrict__ x,
                                                     int64_t nd, double a) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nd; i += (int64_t)gridDim.x * kBlock)
    w[i] = w[i] + a * x[i];
}

// k_trl_coef + k_scale_into in one launch (grid-strided): every block forms
// the same fixed-order sum of the norm partials; block 0 stores alpha/beta,
// all blocks write out = x / ||x|| (zeros for a zero norm).
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_coef_scale(const double* __restrict__ npart, int G,
                                                       const double2* __restrict__ coef, int j,
                                                       double* __restrict__ alpha, double* __restrict__ beta,
                                                       const val_t<VC>* __restrict__ x,
                                                       val_t<VC>* __restrict__ out, int64_t dim,
                                                       int shifted = 0, int jc = -1) {
  double t = 0.0;
  for (int b = threadIdx.x; b < G; b += kBlock) t += npart[b];
  t = block_sum(t);
  const double nrm = sqrt(t);
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    beta[j] = nrm;
    // shifted step (EpiTrlLoc): alpha_j = alpha_{j-1} + <v_j, w>
    const int c = jc >= 0 ? jc : j;
    if (alpha) alpha[j] = shifted ? alpha[j - 1] + coef[c].x : coef[c].x;
  }
  const double inv = nrm > 0.0 ? 1.0 / nrm : 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim; i += (int64_t)gridDim.x * kBlock)
    out[i] = scl(inv, x[i]);
}

// Global-address-space view of a pointer: loads through it are global_load,
// not flat (a flat load also counts against lgkmcnt and waits behind LDS
// traffic).  A no-op for kernel arguments; for pointers read from memory
// (k_trl_batch's task table) the compiler cannot infer it by itself.
template <class T>
__device__ __forceinline__ __attribute__((address_space(1))) T* gptr(T* p) {
  return (__attribute__((address_space(1))) T*)p;
}

// (real vectors only: a class type such as double2 cannot be copied out of
// an address-space-qualified lvalue; the complex callers pass kernel
// arguments, which the compiler already knows to be global)
template <bool VC, class T>
__device__ __forceinline__ auto gptr_real(T* p) {
  if constexpr (VC) return p;
  else return gptr(p);
}

// N wave sums at once (N a multiple of 4): a transposing reduction — each
// v_permlane32_swap / v_permlane16_swap step exchanges half of two values'
// lanes so that one add halves the lanes of both, and the 16-lane rows that
// remain are summed by DPP (4 steps).  ~3 VALU per value per halving for the
// first two levels instead of 18 per value for a full DPP sum each (k_cgs:
// 25 values per wave, ~450 -> ~130 instructions).  Value k lands in row
// {0, 2, 1, 3}[k mod 4] of register k / 4; lane 0 of each row stores it to
// out[k].  Fixed order: deterministic.
__device__ __forceinline__ double swap_add32(double a, double b) {
  // lanes 32-63 of a <-> lanes 0-31 of b; then the lower lanes hold a's two
  // halves' a-values, the upper lanes b's: a' + b' reduces a over lane pairs
  // (l, l+32) in the lower half and b in the upper half
  const auto lo = __builtin_amdgcn_permlane32_swap(__double2loint(a), __double2loint(b), false, false);
  const auto hi = __builtin_amdgcn_permlane32_swap(__double2hiint(a), __double2hiint(b), false, false);
  return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
__device__ __forceinline__ double swap_add16(double a, double b) {
  // odd rows of a <-> even rows of b
  const auto lo = __builtin_amdgcn_permlane16_swap(__double2loint(a), __double2loint(b), false, false);
  const auto hi = __builtin_amdgcn_permlane16_swap(__double2hiint(a), __double2hiint(b), false, false);
  return __hiloint2double(hi[0], lo[0]) + __hiloint2double(hi[1], lo[1]);
}
template <int N>
__device__ __forceinline__ void wave_sum_multi(const double (&v)[N], double* out, int nout) {
  static_assert(N % 4 == 0, "wave_sum_multi: N multiple of 4");
  const int lane = threadIdx.x & 63;
  double t[N / 2];
#pragma unroll
  for (int i = 0; i < N / 2; i++) t[i] = swap_add32(v[2 * i], v[2 * i + 1]);
  double u[N / 4];
#pragma unroll
  for (int i = 0; i < N / 4; i++) {
    double w = swap_add16(t[2 * i], t[2 * i + 1]);
    w = dpp_add<0xB1, 0xF>(w);   // quad_perm [1,0,3,2]
    w = dpp_add<0x4E, 0xF>(w);   // quad_perm [2,3,0,1]
    w = dpp_add<0x141, 0xF>(w);  // row_half_mirror
    w = dpp_add<0x140, 0xF>(w);  // row_mirror: every lane holds its row's sum
    u[i] = w;
  }
  if ((lane & 15) == 0) {
    const int row = lane >> 4;
    const int sub = row == 0 ? 0 : row == 1 ? 2 : row == 2 ? 1 : 3;
#pragma unroll
    for (int i = 0; i < N / 4; i++)
      if (4 * i + sub < nout) out[4 * i + sub] = u[i];
  }
}

// Fused CGS sweep over the rows of x (one column group of up to NC columns
// held in registers per row):
//   hin != nullptr : x_i -= sum_{c<ncol} V_c,i hin_c   (written back)
//   part != nullptr: part[c*G + b] = block partial of <V_c, x> after the update
//   npart != nullptr: npart[b]     = block partial of |x|^2 after the update
// The row loop, the per-thread accumulation order and the subtraction order
// are those of k_vdot_part / k_vaxpy; the block sums use DPP wave sums and one
// barrier for all 2*NC+1 partials.
// (the body takes the launch's block count G and this block's index bx:
// k_cgs passes gridDim.x / blockIdx.x, the lockstep multi-sector solve
// (ed_trlmulti.hpp) its sector's own)
template <bool VC, int NC>
__device__ __forceinline__ void cgs_body(const val_t<VC>* __restrict__ V, int ncol, const double2* __restrict__ hin,
                                         val_t<VC>* __restrict__ x, int64_t dim, double2* __restrict__ part,
                                         double* __restrict__ npart, const double2* __restrict__ pin, int gin,
                                         double2* __restrict__ coef, int add, const double* dgA, const double* dgB,
                                         int* lof, const double* locA, int G, int bx) {
  constexpr int NW = kBlock / 64;
  constexpr int NR = (VC ? 2 * NC : NC) + 1;  // partial slots per wave
  constexpr int NRP = (NR + 3) / 4 * 4;       // padded for wave_sum_multi
  __shared__ double2 hs[NC];
  __shared__ double red[NW][NR];
  // conditional second pass (dgA != null): when the DGKS test says the first
  // pass sufficed, the norm partials of w' (dgB) are this pass's result
  if (dgA && dgks_skip(dgA, dgB, G)) {
    if (threadIdx.x == 0) npart[bx] = dgB[bx];
    return;
  }
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
        if (coef && bx == 0) coef[c] = add ? make_double2(coef[c].x + re, coef[c].y + im) : make_double2(re, im);
      }
    }
    __syncthreads();
  } else if (hin) {
    for (int c = threadIdx.x; c < ncol; c += kBlock) hs[c] = hin[c];
    __syncthreads();
  }
  // first update pass of a fused step (locA = |w|^2 partials of the dots
  // pass): local-only when the far coefficients are noise (cgs_loc_only),
  // its dots then only for the last two columns; the decision goes to *lof
  // for the second pass (the columns it updates)
  int c0 = 0;
  if (locA) {
    const bool lo = cgs_loc_only(hs, ncol, locA, pin ? gin : G);
    if (bx == 0 && threadIdx.x == 0) *lof = lo ? 1 : 0;
    if (lo) c0 = ncol - 2;
  } else if (lof && *lof) {
    c0 = ncol - 2;
  }
  const bool upd = hin || pin;
  const auto Vg = gptr_real<VC>(V);
  const auto xg = gptr_real<VC>(x);
  double are[NC], aim[VC ? NC : 1];
#pragma unroll
  for (int c = 0; c < NC; c++) {
    are[c] = 0.0;
    if constexpr (VC) aim[c] = 0.0;
  }
  double n2 = 0.0;
  // local-only update on real vectors (the common shifted step): two columns
  // and x per row, so the generic loop keeps only ~3 loads in flight per
  // thread; here four rows' loads go out before the first is used (rows
  // still processed in order: the sums are the generic loop's, bit for bit)
  bool loc2 = false;
  double al0 = 0.0, al1 = 0.0;
  if constexpr (!VC) {
    if (upd && c0 > 0 && c0 == ncol - 2) {
      loc2 = true;
      const auto V0 = Vg + (int64_t)c0 * dim;
      const auto V1 = V0 + dim;
      const double h0 = hs[c0].x, h1 = hs[c0 + 1].x;
      const int64_t st = (int64_t)G * kBlock;
      int64_t i = (int64_t)bx * kBlock + threadIdx.x;
      auto row = [&](double a, double b, double xi, int64_t r) {
        xi -= a * h0;
        xi -= b * h1;
        xg[r] = xi;
        if (part) {
          al0 += a * xi;
          al1 += b * xi;
        }
        if (npart) n2 += xi * xi;
      };
      for (; i + 3 * st < dim; i += 4 * st) {
        double a[4], b[4], xv[4];
#pragma unroll
        for (int r = 0; r < 4; r++) {
          a[r] = V0[i + r * st];
          b[r] = V1[i + r * st];
          xv[r] = xg[i + r * st];
        }
#pragma unroll
        for (int r = 0; r < 4; r++) row(a[r], b[r], xv[r], i + r * st);
      }
      for (; i < dim; i += st) row(V0[i], V1[i], xg[i], i);
#pragma unroll
      for (int c = 0; c < NC; c++) are[c] = c == c0 ? al0 : c == c0 + 1 ? al1 : are[c];
    }
  }
  for (int64_t i = (int64_t)bx * kBlock + threadIdx.x; !loc2 && i < dim; i += (int64_t)G * kBlock) {
    val_t<VC> v[NC];
#pragma unroll
    for (int c = 0; c < NC; c++) v[c] = (c >= c0 && c < ncol) ? Vg[(int64_t)c * dim + i] : vzero<val_t<VC>>();
    auto xi = xg[i];
    if (upd) {
#pragma unroll
      for (int c = 0; c < NC; c++) {
        if (c < c0 || c >= ncol) continue;  // uniform
        if constexpr (VC) {
          xi.x -= v[c].x * hs[c].x - v[c].y * hs[c].y;
          xi.y -= v[c].x * hs[c].y + v[c].y * hs[c].x;
        } else {
          xi -= v[c] * hs[c].x;
        }
      }
      xg[i] = xi;
    }
    if (part) {
#pragma unroll
      for (int c = 0; c < NC; c++) {
        if (c < c0) continue;  // uniform (local-only: far dots unused)
        const double2 t = cdotc(v[c], xi);
        are[c] += t.x;
        if constexpr (VC) aim[c] += t.y;
      }
    }
    if (npart) n2 += redot(xi, xi);
  }
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (part) {
    // every dot and the norm in one transposing reduction
    double vals[NRP];
#pragma unroll
    for (int c = 0; c < NRP; c++) vals[c] = 0.0;
#pragma unroll
    for (int c = 0; c < NC; c++) {
      vals[c] = are[c];
      if constexpr (VC) vals[NC + c] = aim[c];
    }
    vals[NR - 1] = n2;
    wave_sum_multi<NRP>(vals, red[wv], NR);
  } else if (npart) {
    const double r = wave_sum_dpp(n2);
    if (lane == 63) red[wv][NR - 1] = r;
  }
  __syncthreads();
  const int t = threadIdx.x;
  if (part && t >= c0 && t < ncol) {
    double re = 0.0, im = 0.0;
#pragma unroll
    for (int w = 0; w < NW; w++) {
      re = re + red[w][t];
      if constexpr (VC) im = im + red[w][NC + t];
    }
    part[(int64_t)t * G + bx] = make_double2(re, im);
  }
  if (npart && t == kBlock - 1) {
    double r = 0.0;
#pragma unroll
    for (int w = 0; w < NW; w++) r = r + red[w][NR - 1];
    npart[bx] = r;
  }
}

template <bool VC, int NC>
__global__ void __launch_bounds__(kBlock) k_cgs(const val_t<VC>* __restrict__ V, int ncol,
                                                const double2* __restrict__ hin,
                                                val_t<VC>* __restrict__ x, int64_t dim,
                                                double2* __restrict__ part, double* __restrict__ npart,
                                                const double2* __restrict__ pin = nullptr, int gin = 0,
                                                double2* __restrict__ coef = nullptr, int add = 0,
                                                const double* dgA = nullptr, const double* dgB = nullptr,
                                                int* lof = nullptr, const double* locA = nullptr) {
  cgs_body<VC, NC>(V, ncol, hin, x, dim, part, npart, pin, gin, coef, add, dgA, dgB, lof, locA, (int)gridDim.x,
                   (int)blockIdx.x);
}

// ------------------------------------------------------------------------
// Whole orthogonalisation of one Krylov step in ONE workgroup (sectors up to
// kOrthSoloMaxDim rows).  The multi-kernel form is three k_cgs launches and a
// k_coef_scale (each a few microseconds of launch and latency on a sector
// of a few hundred rows: ~30 of the ~36 us a small-sector step took).  Here
// the block does CGS pass 1 (dots, |x|^2), pass 2 (x -= V h1, dots, |x'|^2),
// the DGKS test, the conditional pass 3 (x -= V h2, |x''|^2), alpha/beta and
// V_{j+1} = x / beta with block reductions between the passes: a Krylov step
// is the H·v and this launch.  Same coefficients, same test, same semantics
// as Trlan::orth's fused sweeps (coef = h1, + h2 when the second pass runs;
// beta[jslot] = |x|; alpha[jn] when jn >= 0, shifted by alpha[jn-1] after an
// EpiTrlLoc product).
constexpr int kOrthSoloBlock = 512;
constexpr int64_t kOrthSoloMaxDim = 2048;  // measured: dim 2,640 35 us per step solo, 31 multi-kernel

template <bool VC, int NC, int RU = 1>
__device__ __forceinline__ void orth_solo_body(const val_t<VC>* __restrict__ V, int ncol,
                                               val_t<VC>* __restrict__ x, int64_t dim,
                                               double2* __restrict__ coef, double* __restrict__ alpha,
                                               double* __restrict__ beta, int jn, int jslot,
                                               val_t<VC>* __restrict__ out, int shifted, int locupd,
                                               int jc = -1) {
  using Vt = val_t<VC>;
  if (jc < 0) jc = jn;
  const auto Vg = gptr_real<VC>(V);
  const auto xg = gptr_real<VC>(x);  // basis column of v_j (alpha slot jn)
  constexpr int NT = kOrthSoloBlock, NW = NT / 64;
  constexpr int NR = (VC ? 2 * NC : NC) + 1;  // partial slots: re[NC] | im[NC] | norm
  __shared__ double red[NW][NR];
  __shared__ double tot[NR];
  __shared__ double2 h1[NC], h2[NC];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  double are[NC], aim[VC ? NC : 1];
  // block sums (fixed order): are/aim (first nc columns) and n2 -> tot
  auto reduce = [&](int nc, double n2) {
    if (nc >= 4) {  // uniform: every value in one transposing reduction
      constexpr int NRP = (NR + 3) / 4 * 4;
      double vals[NRP];
#pragma unroll
      for (int c = 0; c < NRP; c++) vals[c] = 0.0;
#pragma unroll
      for (int c = 0; c < NC; c++) {
        vals[c] = are[c];
        if constexpr (VC) vals[NC + c] = aim[c];
      }
      vals[NR - 1] = n2;
      wave_sum_multi<NRP>(vals, red[wv], NR);
    } else {
#pragma unroll
      for (int c = 0; c < NC; c++) {
        if (c >= nc) continue;  // uniform
        const double r = wave_sum_dpp(are[c]);
        if (lane == 63) red[wv][c] = r;
        if constexpr (VC) {
          const double q = wave_sum_dpp(aim[c]);
          if (lane == 63) red[wv][NC + c] = q;
        }
      }
      const double r = wave_sum_dpp(n2);
      if (lane == 63) red[wv][NR - 1] = r;
    }
    __syncthreads();
    if (t < NR) {
      double a = 0.0;
#pragma unroll
      for (int w = 0; w < NW; w++) a = a + red[w][t];
      tot[t] = a;
    }
    __syncthreads();
  };
  auto zero = [&]() {
#pragma unroll
    for (int c = 0; c < NC; c++) {
      are[c] = 0.0;
      if constexpr (VC) aim[c] = 0.0;
    }
  };
  // one row: x_i -= V_i h (written back), dots, |x_i|^2
  auto row = [&](const Vt (&v)[NC], Vt xi, int64_t i, const double2* h, bool dots, int c0, double& n2) {
    {
      if (h) {
#pragma unroll
        for (int c = 0; c < NC; c++) {
          if (c < c0 || c >= ncol) continue;  // uniform
          if constexpr (VC) {
            xi.x -= v[c].x * h[c].x - v[c].y * h[c].y;
            xi.y -= v[c].x * h[c].y + v[c].y * h[c].x;
          } else {
            xi -= v[c] * h[c].x;
          }
        }
        xg[i] = xi;
      }
      if (dots) {
#pragma unroll
        for (int c = 0; c < NC; c++) {
          const double2 d = cdotc(v[c], xi);
          are[c] += d.x;
          if constexpr (VC) aim[c] += d.y;
        }
      }
      n2 += redot(xi, xi);
    }
  };
  auto pass = [&](const double2* h, bool dots, int c0) {
    double n2 = 0.0;
    int64_t i = t;
    if constexpr (RU == 2) {
      // two rows' loads in flight before either is used (one workgroup on a
      // few thousand rows is bound by the load latency of each row); rows
      // still processed in order, so the sums are those of the plain loop
      for (; i + NT < dim; i += 2 * NT) {
        Vt va[NC], vb[NC];
#pragma unroll
        for (int c = 0; c < NC; c++) {
          const bool on = c >= c0 && c < ncol;
          va[c] = on ? Vg[(int64_t)c * dim + i] : vzero<Vt>();
          vb[c] = on ? Vg[(int64_t)c * dim + i + NT] : vzero<Vt>();
        }
        const Vt xa = xg[i], xb = xg[i + NT];
        row(va, xa, i, h, dots, c0, n2);
        row(vb, xb, i + NT, h, dots, c0, n2);
      }
    }
    for (; i < dim; i += NT) {
      Vt v[NC];
#pragma unroll
      for (int c = 0; c < NC; c++) v[c] = (c >= c0 && c < ncol) ? Vg[(int64_t)c * dim + i] : vzero<Vt>();
      row(v, xg[i], i, h, dots, c0, n2);
    }
    return n2;
  };  // x -= V[:, c0:ncol] h (h in LDS); optional dots of the result; returns |x|^2 partial
  // pass 1: h1 = V^H x, |x|^2
  zero();
  reduce(ncol, pass(nullptr, true, 0));
  const double nA = tot[NR - 1];
  if (t < ncol) h1[t] = make_double2(tot[t], VC ? tot[NC + t] : 0.0);
  __syncthreads();
  // local-only update (kCgsLocTol): passes 2 and 3 on the last two columns
  const int c0 = (locupd && cgs_loc_only(h1, ncol, tot + (NR - 1), 1)) ? ncol - 2 : 0;
  // pass 2: x -= V h1; h2 = V^H x, |x'|^2
  zero();
  reduce(ncol, pass(h1, true, c0));
  const double nB = tot[NR - 1];
  if (t < ncol) h2[t] = make_double2(tot[t], VC ? tot[NC + t] : 0.0);  // (far: 0 when local-only)
  __syncthreads();
  double nF = nB;
  const bool second = !(nB > kDgks2 * nA);  // ARPACK's DGKS test (block-uniform)
  if (second) {
    zero();
    reduce(0, pass(h2, false, c0));
    nF = tot[NR - 1];
  }
  if (t < ncol) {
    const double2 c = second ? make_double2(h1[t].x + h2[t].x, h1[t].y + h2[t].y) : h1[t];
    coef[t] = c;
    if (t == jc && jn >= 0 && alpha) alpha[jn] = shifted ? alpha[jn - 1] + c.x : c.x;
  }
  const double b = sqrt(nF);
  if (t == 0) beta[jslot] = b;
  if (out) {
    const double inv = b > 0.0 ? 1.0 / b : 0.0;
    const auto og = gptr_real<VC>(out);
    for (int64_t i = t; i < dim; i += NT) og[i] = scl(inv, xg[i]);
  }
}

template <bool VC, int NC>
__global__ void __launch_bounds__(kOrthSoloBlock) k_orth_solo(const val_t<VC>* __restrict__ V, int ncol,
                                                              val_t<VC>* __restrict__ x, int64_t dim,
                                                              double2* __restrict__ coef, double* __restrict__ alpha,
                                                              double* __restrict__ beta, int jn, int jslot,
                                                              val_t<VC>* __restrict__ out, int shifted,
                                                              int locupd, int jc) {
  orth_solo_body<VC, NC>(V, ncol, x, dim, coef, alpha, beta, jn, jslot, out, shifted, locupd, jc);
}

// A whole Krylov step of a small stored sector in ONE workgroup (real
// vectors, packed SELL words): v_j staged in LDS, H v_j gathered from LDS
// with the shifted three-term epilogue (EpiTrlLoc's arithmetic when
// shifted), then orth_solo_body.  The sweep is one launch per step instead
// of two (the H·v grid and k_orth_solo).  Same per-row sums as k_spmv_pk.
struct StepSoloArgs {
  const double* diag;
  const int64_t* sptr;
  const uint32_t* words;
  const double* dict;  // 256 entries
  const double* Vb;    // basis, column c at Vb + c*dim
  double* x;           // w (the step's residual)
  double* out;         // V_{j+1} = w / beta_j, or null (last column of the sweep)
  double2* coef;
  double* alpha;
  double* beta;
  int64_t dim;
  int j, shifted;      // column j; shifted: w = (H - alpha_{j-1}) v_j - beta_{j-1} v_{j-1}
  int locupd;          // local-only CGS update allowed (kCgsLocTol)
};

template <int NC>
__global__ void __launch_bounds__(kOrthSoloBlock) k_step_solo(const StepSoloArgs a) {
  constexpr int NT = kOrthSoloBlock;
  __shared__ double vl[kOrthSoloMaxDim];
  __shared__ double sdict[256];
  const int t = threadIdx.x;
  const int64_t dim = a.dim;
  const int j = a.j;
  const double* vj = a.Vb + (int64_t)j * dim;
  for (int64_t i = t; i < dim; i += NT) vl[i] = vj[i];
  if (t < 256) sdict[t] = a.dict[t];
  double sg = 0.0, bp = 0.0;
  if (a.shifted) {
    sg = a.alpha[j - 1];
    bp = a.beta[j - 1];
  }
  __syncthreads();
  const double* vprev = a.shifted ? a.Vb + (int64_t)(j - 1) * dim : nullptr;
  for (int64_t i = t; i < dim; i += NT) {
    const int64_t sl = i >> 6, s0 = a.sptr[sl];
    const int w = (int)((a.sptr[sl + 1] - s0) >> 6);
    const uint32_t* wp = a.words + s0 + (i & 63);
    const double xi = vl[i];
    double acc = 0.0 + a.diag[i] * xi;
    for (int k0 = 0; k0 < w; k0 += kChunk) {
      uint32_t c[kChunk];
#pragma unroll
      for (int k = 0; k < kChunk; k++) c[k] = (k0 + k < w) ? wp[64 * (k0 + k)] : (uint32_t)i;
#pragma unroll
      for (int k = 0; k < kChunk; k++)
        if (k0 + k < w) acc = acc + sdict[c[k] >> kPackShift] * vl[c[k] & kPackColMask];
    }
    a.x[i] = a.shifted ? (acc - sg * xi) - bp * vprev[i] : acc;
  }
  // (each thread's orthogonalisation passes read back only its own rows of x)
  orth_solo_body<false, NC>(a.Vb, j + 1, a.x, dim, a.coef, a.alpha, a.beta, j, j, a.out, a.shifted,
                            a.shifted && a.locupd);
}


}  // namespace edg
