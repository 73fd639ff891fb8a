// ed_kernels.hpp — HIP kernels of the H·v hot path for gfx950 (CDNA4).
//
// Kernels (one thread per basis row, 256-thread blocks = 4 wavefronts,
// grid-strided over whole 64-row slices so that a wavefront is exactly one
// SELL slice):
//   k_build_map    H%map from the (off, rank) tables        build_sector ED_SETUP.f90:886-984
//   k_count        elements per row + SELL-64 slice width   ed_buildH_c pass 1
//   k_fill         SELL-64 fill, reference row order        ed_buildH_c + sp_insert_element
//   k_spmv         stored H·v, SELL-64                      spMatVec_cc STORED_HxV.f90:132-143
//   k_spmv_pk      same, 32-bit {col|dictionary index} words (real H)
//   k_direct       matrix-free H·v (gather, any ed_mode)     directMatVec_cc DIRECT_HxV.f90:21-92
//   k_kron         matrix-free H·v, normal mode without Jx/Jp: H = D + Hup(x)1 + 1(x)Hdw
//   k_lanc_*       device-resident plain Lanczos recurrence .repo/PLAIN_LANCZOS.f90:87-118
//
// The three H·v kernels share one epilogue interface, so the Lanczos update
// (w = Hv - b*v_prev, alpha = <v,w>) is fused into the H·v pass and the
// partial dot products are combined in-kernel by the last block to finish
// (deterministic fixed-order sum, agent-scope release/acquire per
// cdna_hip_programming.md Guideline 16).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

#include "ed_model.hpp"

namespace edg {

constexpr int kBlock = 256;  // 4 wavefronts of 64

// ------------------------------------------------------------------ values
template <bool C> using val_t = typename std::conditional<C, double2, double>::type;

__device__ __forceinline__ double mkval(double re, double, std::false_type) { return re; }
__device__ __forceinline__ double2 mkval(double re, double im, std::true_type) { return make_double2(re, im); }
template <bool C> __device__ __forceinline__ val_t<C> mk(double re, double im) {
  return mkval(re, im, std::integral_constant<bool, C>());
}

__device__ __forceinline__ double mul(double h, double x) { return h * x; }
__device__ __forceinline__ double2 mul(double h, double2 x) { return make_double2(h * x.x, h * x.y); }
__device__ __forceinline__ double2 mul(double2 h, double2 x) {
  return make_double2(h.x * x.x - h.y * x.y, h.x * x.y + h.y * x.x);
}
// acc + h*x with fused multiply-adds (persistent register paths only: the
// stored/direct H·v kernels keep separate mul/add for bit-parity with the
// oracle's spMatVec_cc)
__device__ __forceinline__ double fmac(double acc, double h, double x) { return __fma_rn(h, x, acc); }
__device__ __forceinline__ double2 fmac(double2 acc, double h, double2 x) {
  return make_double2(__fma_rn(h, x.x, acc.x), __fma_rn(h, x.y, acc.y));
}
__device__ __forceinline__ double2 fmac(double2 acc, double2 h, double2 x) {
  return make_double2(__fma_rn(-h.y, x.y, __fma_rn(h.x, x.x, acc.x)), __fma_rn(h.y, x.x, __fma_rn(h.x, x.y, acc.y)));
}
__device__ __forceinline__ double add(double a, double b) { return a + b; }
__device__ __forceinline__ double2 add(double2 a, double2 b) { return make_double2(a.x + b.x, a.y + b.y); }
__device__ __forceinline__ double sub(double a, double b) { return a - b; }
__device__ __forceinline__ double2 sub(double2 a, double2 b) { return make_double2(a.x - b.x, a.y - b.y); }
__device__ __forceinline__ double scl(double s, double a) { return s * a; }
__device__ __forceinline__ double2 scl(double s, double2 a) { return make_double2(s * a.x, s * a.y); }
// component-wise select (a ternary on the double2 struct goes through
// scratch memory: 5x slower complex SpMV)
__device__ __forceinline__ double sel(bool c, double a, double b) { return c ? a : b; }
__device__ __forceinline__ double2 sel(bool c, double2 a, double2 b) {
  return make_double2(c ? a.x : b.x, c ? a.y : b.y);
}
__device__ __forceinline__ double re_of(double a) { return a; }
__device__ __forceinline__ double re_of(double2 a) { return a.x; }
// Re(conj(a)*b): dot_product real part
__device__ __forceinline__ double redot(double a, double b) { return a * b; }
__device__ __forceinline__ double redot(double2 a, double2 b) { return a.x * b.x + a.y * b.y; }
template <class V> __device__ __forceinline__ V vzero();
template <> __device__ __forceinline__ double vzero<double>() { return 0.0; }
template <> __device__ __forceinline__ double2 vzero<double2>() { return make_double2(0.0, 0.0); }

// -------------------------------------------------------------- reductions
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = max(v, __shfl_xor(v, o, 64));
  return v;
}
// Deterministic block sum over NT threads; result valid in every thread.
template <int NT = kBlock>
__device__ __forceinline__ double block_sum(double v) {
  __shared__ double ws[NT / 64];
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = v;
  __syncthreads();
  double t = 0.0;
#pragma unroll
  for (int w = 0; w < NT / 64; w++) t = t + ws[w];
  return t;
}

struct RedSlot {
  double* partials;       // [gridDim.x]
  unsigned int* counter;  // zero on entry; reset by the last block.  nullptr:
                          // two-pass mode (plain partial stores, a one-block
                          // finishing kernel sums them after the boundary)
};

// Largest grid that finishes its reduction in-kernel: one ticket word takes
// ~88 atomics/us (MI355X_MICROARCH.md, row "dequeue"), so thousands of blocks
// would serialise on it; beyond this the finishing kernel is cheaper.
constexpr int kTicketMaxBlocks = 128;

// Two-pass mode, pass 1: block partial -> partials[blockIdx.x].
template <int NT = kBlock>
__device__ __forceinline__ void block_partial(double v, double* partials) {
  double s = block_sum<NT>(v);
  if (threadIdx.x == 0) partials[blockIdx.x] = s;
}
// Pass 2 (one 256-thread block): the same fixed-order sum as grid_reduce_last.
__device__ __forceinline__ double sum_partials(const double* partials, int n) {
  double a = 0.0;
  for (int b = threadIdx.x; b < n; b += kBlock) a = a + partials[b];
  return block_sum(a);
}

// Block-partial sum -> partials; the last block to arrive (atomic ticket)
// returns true with the full sum in *total (fixed order: independent of
// arrival order).
//
// Hand-off protocol (MI355X_MICROARCH.md, "Valid forms", first table row):
// one lane per block stores its partial write-through (relaxed agent-scope
// atomic store = global_store ... sc1), drains it with s_waitcnt vmcnt(0),
// then takes a ticket with an agent-scope atomic add; the block whose add
// returns gridDim-1 reads every partial with sc1 loads (relaxed agent-scope
// atomic loads) after a workgroup barrier.  No release/acquire fence: a
// release fence (buffer_wbl2) per block writes back the XCD L2's dirty lines
// and, with thousands of blocks that just wrote H·v outputs, serialises the
// kernel (measured 7x slower Lanczos steps on the c4 sector).
template <int NT = kBlock>
__device__ __forceinline__ bool grid_reduce_last(double v, RedSlot slot, double* total) {
  __shared__ int amlast;
  // every storing wave drains its (write-through) stores before the block's
  // ticket (R1: the signalling lane signals behind a workgroup barrier)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  double s = block_sum<NT>(v);
  if (threadIdx.x == 0) {
    __hip_atomic_store(slot.partials + blockIdx.x, s, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    unsigned int t = __hip_atomic_fetch_add(slot.counter, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    amlast = (t == gridDim.x - 1);
  }
  __syncthreads();
  if (!amlast) return false;
  double a = 0.0;
  for (unsigned int b = threadIdx.x; b < gridDim.x; b += NT)
    a = a + __hip_atomic_load(slot.partials + b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  *total = block_sum<NT>(a);
  if (threadIdx.x == 0) *slot.counter = 0u;
  return true;
}

// ---------------------------------------------------------------- indexing
struct DevIndex {
  const int32_t* off;
  const uint32_t* rank;
  int ns;
  uint32_t mask;
  __device__ __forceinline__ int32_t operator()(uint32_t k) const {
    return off[k >> ns] + (int32_t)rank[k & mask];
  }
};

// ------------------------------------------------------------- basis / map
static __global__ void __launch_bounds__(kBlock) k_build_map(const int64_t* __restrict__ blk_off,
                                                      const uint32_t* __restrict__ blk_idw, int nblk,
                                                      const int32_t* __restrict__ need_cls,
                                                      const uint32_t* __restrict__ by_cls,
                                                      const int32_t* __restrict__ cls_start, int ns,
                                                      int64_t dim, uint32_t* __restrict__ map) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim;
       i += (int64_t)gridDim.x * kBlock) {
    int lo = 0, hi = nblk;  // blk_off[lo] <= i < blk_off[hi]
    while (hi - lo > 1) {
      int mid = (lo + hi) >> 1;
      if (blk_off[mid] <= i) lo = mid;
      else hi = mid;
    }
    uint32_t idw = blk_idw[lo];
    uint32_t iup = by_cls[cls_start[need_cls[idw]] + (i - blk_off[lo])];
    map[i] = iup | (idw << ns);
  }
}

// ------------------------------------------------------------ stored build
struct CountAcc {
  int n = 0;
  __device__ __forceinline__ void diag(double, double) {}
  __device__ __forceinline__ void off(uint32_t, double, double) { n++; }
};

// cnt[i] = off-diagonal elements of row i; width[s] = max over slice s.
static __global__ void __launch_bounds__(kBlock) k_count(const EdModel* __restrict__ Mp,
                                                  const uint32_t* __restrict__ map, int64_t dim,
                                                  int64_t nslice, uint16_t* __restrict__ cnt,
                                                  int32_t* __restrict__ width) {
  const EdModel& M = *Mp;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nslice * 64;
       i += (int64_t)gridDim.x * kBlock) {
    int c = 0;
    if (i < dim) {
      CountAcc a;
      gen_row(M, map[i], a);
      c = a.n;
      cnt[i] = (uint16_t)c;
    }
    int w = wave_max(c);
    if ((threadIdx.x & 63) == 0) width[i >> 6] = w;
  }
}

// Exclusive scan of 64*width -> sptr (int64), three-pass.
// *out += sum of n 16-bit counts (grid-strided; wave sums, one atomic per wave)
static __global__ void __launch_bounds__(kBlock) k_sum_u16(const uint16_t* __restrict__ c, int64_t n,
                                                    unsigned long long* out) {
  unsigned long long acc = 0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) acc += c[i];
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(out, acc);
}

static __global__ void __launch_bounds__(1024) k_scan_blocks(const int32_t* __restrict__ width, int64_t n,
                                                      int64_t* __restrict__ out,
                                                      int64_t* __restrict__ bsum) {
  __shared__ int64_t s[1024];
  int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  int64_t x = (i < n) ? 64 * (int64_t)width[i] : 0;
  s[threadIdx.x] = x;
  __syncthreads();
  for (int o = 1; o < 1024; o <<= 1) {
    int64_t t = (threadIdx.x >= (unsigned)o) ? s[threadIdx.x - o] : 0;
    __syncthreads();
    s[threadIdx.x] += t;
    __syncthreads();
  }
  if (i < n) out[i] = s[threadIdx.x] - x;  // exclusive within block
  if (threadIdx.x == 1023) bsum[blockIdx.x] = s[1023];
}
static __global__ void k_scan_spine(int64_t* __restrict__ bsum, int64_t nb, int64_t* __restrict__ total) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    int64_t acc = 0;
    for (int64_t b = 0; b < nb; b++) {
      int64_t t = bsum[b];
      bsum[b] = acc;
      acc += t;
    }
    *total = acc;
  }
}
static __global__ void __launch_bounds__(1024) k_scan_add(int64_t* __restrict__ out, int64_t n,
                                                   const int64_t* __restrict__ bsum,
                                                   const int64_t* __restrict__ total) {
  int64_t i = (int64_t)blockIdx.x * 1024 + threadIdx.x;
  if (i < n) out[i] += bsum[blockIdx.x];
  if (i == 0) out[n] = *total;
}

template <bool HC>
struct FillAcc {
  using H = val_t<HC>;
  int64_t base;
  int k = 0;
  DevIndex idx;
  int32_t* cols;
  H* vals;
  H dv;
  __device__ __forceinline__ void diag(double re, double im) { dv = mk<HC>(re, im); }
  __device__ __forceinline__ void off(uint32_t kst, double re, double im) {
    int64_t q = base + 64 * (int64_t)k;
    cols[q] = idx(kst);
    vals[q] = mk<HC>(re, im);
    k++;
  }
};

template <bool HC>
__global__ void __launch_bounds__(kBlock) k_fill(const EdModel* __restrict__ Mp,
                                                 const uint32_t* __restrict__ map, int64_t dim,
                                                 DevIndex idx, const int64_t* __restrict__ sptr,
                                                 val_t<HC>* __restrict__ diag,
                                                 int32_t* __restrict__ cols,
                                                 val_t<HC>* __restrict__ vals) {
  const EdModel& M = *Mp;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim;
       i += (int64_t)gridDim.x * kBlock) {
    int64_t s = i >> 6;
    FillAcc<HC> a;
    a.base = sptr[s] + (i & 63);
    a.idx = idx;
    a.cols = cols;
    a.vals = vals;
    gen_row(M, map[i], a);
    diag[i] = a.dv;
    int w = (int)((sptr[s + 1] - sptr[s]) >> 6);
    for (int k = a.k; k < w; k++) {  // padding: own column, zero value
      int64_t q = a.base + 64 * (int64_t)k;
      cols[q] = (int32_t)i;
      vals[q] = mk<HC>(0.0, 0.0);
    }
  }
  // lanes past dim in the last slice: defined padding too (every slot of the
  // SELL arrays is then a valid (col, value) pair, e.g. for the packed form)
  const int64_t tail = ((dim + 63) & ~(int64_t)63) - dim;
  if (blockIdx.x == 0 && threadIdx.x < tail) {
    const int64_t i = dim + threadIdx.x, s = i >> 6;
    const int w = (int)((sptr[s + 1] - sptr[s]) >> 6);
    for (int k = 0; k < w; k++) {
      const int64_t q = sptr[s] + (i & 63) + 64 * (int64_t)k;
      cols[q] = 0;
      vals[q] = mk<HC>(0.0, 0.0);
    }
  }
}

// --------------------------------------------------------------- epilogues
// row(i, acc, xi) receives (H x)_i and x_i; returns the row's contribution to
// the fused reduction.  finish(part) runs once per thread after the loop.
template <bool VC>
struct EpiStore {
  using V = val_t<VC>;
  V* hv;
  V* scratch() const { return hv; }  // where a two-pass H·v puts its first pass
  __device__ __forceinline__ bool skip() const { return false; }
  __device__ __forceinline__ void prepare() {}
  // non-temporal: the Hv stream evicts fewer of the gathered vector's lines
  // from L2 (same-process A/B at N28: stored complex 0.364 -> 0.350 ms,
  // k_direct 0.170 -> 0.164 ms, stored real neutral)
  __device__ __forceinline__ double row(int64_t i, V acc, V) {
    if constexpr (VC) {
      typedef double d2 __attribute__((ext_vector_type(2)));
      __builtin_nontemporal_store(d2{acc.x, acc.y}, (d2*)(hv + i));
    } else {
      __builtin_nontemporal_store(acc, hv + i);
    }
    return 0.0;
  }
  template <int NT = kBlock>
  __device__ __forceinline__ void finish(double) {}
};

// Thick-restart Lanczos step j past a restart (Trlan::step, ed_lib.hip):
// the three-term part of the recurrence is applied as H v_j is stored, with
// the spectral shift sigma = alpha_{j-1},
//   w = (H - sigma) v_j - beta_{j-1} v_{j-1}
// (alpha_j = sigma + <v_j, w>, k_coef_scale).  The Gram-Schmidt pass then
// meets only the remainder: ARPACK's DGKS test (||w'|| > 0.717 ||w||, which
// bounds the growth of the basis' orthogonality error) passes whenever
// |alpha_j - alpha_{j-1}| < 0.97 beta_j, and the second pass over the basis
// is skipped.  On the raw w = H v_j the test can never pass (w carries
// beta_{j-1} v_{j-1} and alpha_j v_j: ||w'|| / ||w|| < 1/sqrt(2)).
template <bool VC>
struct EpiTrlLoc {
  using V = val_t<VC>;
  V* hv;
  const V* vprev;        // v_{j-1}
  const double* sig;     // &alpha[j-1]
  const double* bprev;   // &beta[j-1]
  double s = 0.0, b = 0.0;
  V* scratch() const { return hv; }
  __device__ __forceinline__ bool skip() const { return false; }
  __device__ __forceinline__ void prepare() {
    s = *sig;
    b = *bprev;
  }
  __device__ __forceinline__ double row(int64_t i, V acc, V xi) {
    hv[i] = sub(sub(acc, scl(s, xi)), scl(b, vprev[i]));
    return 0.0;
  }
  template <int NT = kBlock>
  __device__ __forceinline__ void finish(double) {}
};

// Device scalars of one Lanczos run.
struct LancState {
  double beta;    // b of the previous iteration (normalisation of R)
  double invb;    // 1/b
  double alpha;   // a of the current iteration
  double thresh;  // breakdown threshold
  double tmp;
  int iter;       // iterations completed
  int done;       // breakdown reached
  int pad[2];
};

// Lanczos step, part A (fused into the H·v kernel).  Input R = unnormalised
// r_k (b_k = st->beta), P = v_{k-1}.  Per row: v = R*invb, w = (H R)*invb - b*P,
// P <- v, W <- w; alpha_k = sum Re(conj(v) w).  .repo/PLAIN_LANCZOS.f90:105-114
template <bool VC>
struct EpiLancA {
  using V = val_t<VC>;
  LancState* st;
  V* P;
  V* W;
  V* basis;      // optional: Krylov basis, column k at basis + k*dim
  int64_t dim;
  double* alpha_out;
  RedSlot slot;
  double invb, b;
  V* bcol;
  V* scratch() const { return W; }  // W is rewritten row by row by row() itself
  __device__ __forceinline__ bool skip() const { return st->done != 0; }
  __device__ __forceinline__ void prepare() {
    invb = st->invb;
    b = st->beta;
    bcol = basis ? basis + (int64_t)st->iter * dim : nullptr;
  }
  __device__ __forceinline__ double row(int64_t i, V acc, V xi) {
    V v = scl(invb, xi);
    V h = scl(invb, acc);
    V w = sub(h, scl(b, P[i]));
    P[i] = v;
    W[i] = w;
    if (bcol) bcol[i] = v;
    return redot(v, w);
  }
  template <int NT = kBlock>
  __device__ __forceinline__ void finish(double part) {
    if (!slot.counter) {
      block_partial<NT>(part, slot.partials);
      return;
    }
    double tot;
    if (grid_reduce_last<NT>(part, slot, &tot) && threadIdx.x == 0) {
      st->alpha = tot;
      alpha_out[st->iter] = tot;
    }
  }
};

// sc1 (write-through, L1-bypassing) element stores / loads for vectors handed
// from every block to the last block of the same kernel.
__device__ __forceinline__ void st_wt(double* p, double v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ void st_wt(double2* p, double2 v) {
  __hip_atomic_store((double*)p, v.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  __hip_atomic_store((double*)p + 1, v.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_wt(const double* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double2 ld_wt(const double2* p) {
  return make_double2(__hip_atomic_load((const double*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT),
                      __hip_atomic_load((const double*)p + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

// Two-pass finishing kernels of one Lanczos step (one block of kBlock threads).
static __global__ void __launch_bounds__(kBlock) k_lanc_fin_a(const double* __restrict__ partials, int n,
                                                       LancState* st, double* alpha_out) {
  if (st->done) return;
  const double tot = sum_partials(partials, n);
  if (threadIdx.x == 0) {
    st->alpha = tot;
    alpha_out[st->iter] = tot;
  }
}
__device__ __forceinline__ void lanc_set_beta(double tot, LancState* st, double* beta_out) {
  const double b = sqrt(tot);
  const int it = st->iter;
  beta_out[it + 1] = b;
  st->beta = b;
  st->invb = 1.0 / b;
  st->iter = it + 1;
  if (b < st->thresh) st->done = 1;
}
static __global__ void __launch_bounds__(kBlock) k_lanc_fin_b(const double* __restrict__ partials, int n,
                                                       LancState* st, double* beta_out) {
  if (st->done) return;
  const double tot = sum_partials(partials, n);
  if (threadIdx.x == 0) lanc_set_beta(tot, st, beta_out);
}

// ------------------------------------------------------------- stored H·v
// Matrix-stream loads; NT=1 marks them non-temporal (used when the matrix does
// not fit the 256 MB Infinity Cache, so caching it only evicts v).
template <int NT, class T>
__device__ __forceinline__ T ldm(const T* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int NT>
__device__ __forceinline__ double2 ldm2(const double2* p) {
  if constexpr (NT) {
    const double* q = (const double*)p;
    return make_double2(__builtin_nontemporal_load(q), __builtin_nontemporal_load(q + 1));
  } else {
    return *p;
  }
}
template <int NT> __device__ __forceinline__ double ldh(const double* p) { return ldm<NT>(p); }
template <int NT> __device__ __forceinline__ double2 ldh(const double2* p) { return ldm2<NT>(p); }

// One thread per row; the row's entries are fetched in chunks of kChunk with
// every column and value load of a chunk issued before the gathers (measured
// +10-14 % over a plain loop on the Nlevels=28 sector), summed in row order.
constexpr int kChunk = 16;

template <bool HC, bool VC, int NT, class Epi>
__global__ void __launch_bounds__(kBlock) k_spmv(const val_t<HC>* __restrict__ diag,
                                                 const int64_t* __restrict__ sptr,
                                                 const int32_t* __restrict__ cols,
                                                 const val_t<HC>* __restrict__ vals,
                                                 const val_t<VC>* __restrict__ x,
                                                 const val_t<VC>* __restrict__ xr, int64_t dim,
                                                 int64_t nslice, Epi epi, int xcd) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  if (epi.skip()) return;
  epi.prepare();
  double part = 0.0;
  auto body = [&](int64_t i) {
    {
      const int64_t s = (int64_t)__builtin_amdgcn_readfirstlane((int)(i >> 6));  // wave-uniform (k_spmv_pk)
      const int64_t s0 = sptr[s];
      const int w = (int)((sptr[s + 1] - s0) >> 6);
      const int32_t* cp = cols + s0 + (i & 63);
      const H* vp = vals + s0 + (i & 63);
      const V xi = xr[i];  // own entry: xr = x + first row (row-split sectors)
      // spMatVec_cc: Hv=0; Hv(i)=Hv(i)+vals(j)*v(cols(j)), diagonal first
      V acc = add(vzero<V>(), mul(ldh<NT>(diag + i), xi));
      for (int k0 = 0; k0 < w; k0 += kChunk) {
        int32_t c[kChunk];
        H h[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; k++) c[k] = (k0 + k < w) ? ldm<NT>(cp + 64 * (k0 + k)) : (int32_t)i;
#pragma unroll
        for (int k = 0; k < kChunk; k++)
          h[k] = (k0 + k < w) ? ldh<NT>(vp + 64 * (k0 + k)) : mk<HC>(0.0, 0.0);
        V g[kChunk];
#pragma unroll
        for (int k = 0; k < kChunk; k++) g[k] = x[c[k]];
#pragma unroll
        for (int k = 0; k < kChunk; k++)
          if (k0 + k < w) acc = add(acc, mul(h[k], g[k]));
      }
      part += epi.row(i, acc, xi);
    }
  };
  {
    // one row range per XCD (see k_spmv_pk)
    int64_t b = blockIdx.x;
    if (xcd) b = (b & 7) * (gridDim.x >> 3) + (b >> 3);
    for (int64_t i = b * kBlock + threadIdx.x; i < nslice * 64; i += (int64_t)gridDim.x * kBlock)
      if (i < dim) body(i);
  }
  epi.finish(part);
}

// ------------------------------------------- stored H·v, packed (real H)
// When a real sector's off-diagonal values take at most 256 distinct bit
// patterns (hoppings, exchange, pair hopping: tens), each SELL slot is one
// 32-bit word {col:24 | dictionary index:8}: 4 B per entry instead of 12,
// the value read from a 2 KB dictionary that stays in L1.  Same slots, same
// order, same doubles as k_spmv: bit-identical results.
constexpr int kPackShift = 24;
constexpr uint32_t kPackColMask = (1u << kPackShift) - 1;
constexpr int kDictTable = 4096;  // open-addressing hash of value bit patterns
constexpr unsigned long long kDictEmpty = ~0ull;

__device__ __forceinline__ uint32_t dict_hash(unsigned long long k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  return (uint32_t)k & (kDictTable - 1);
}

// Insert every value's bit pattern; plain reads first so that the few
// distinct keys cost one CAS each, not one per slot.
// Wave-level deduplication before the table: the lanes of a wavefront read 64
// consecutive SELL slots, which hold only a few distinct values (hoppings);
// one leader per distinct key goes to the table.  Without it every slot did a
// read (and the first ones a CAS) of the same few table lines: all of the
// device's requests on one L2 channel (N28: 1.05 ms; c4 farm: 0.75 ms per
// sector, 0.125 s of the serial configs[3] farm).
__device__ __forceinline__ bool wave_key_leader(unsigned long long key) {
  const int lane = threadIdx.x & 63;
  unsigned long long pending = __ballot(1);
  bool lead = false;
  while (pending) {
    const int l = __ffsll((long long)pending) - 1;
    const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)key, l);
    const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(key >> 32), l);
    const unsigned long long kl = ((unsigned long long)hi << 32) | lo;
    const unsigned long long same = __ballot(key == kl);
    lead |= lane == l;
    pending &= ~same;
  }
  return lead;
}

static __global__ void __launch_bounds__(kBlock) k_dict_insert(const double* __restrict__ vals, int64_t n,
                                                        unsigned long long* table,
                                                        unsigned int* overflow) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const unsigned long long key = (unsigned long long)__double_as_longlong(vals[i]);
    if (!wave_key_leader(key)) continue;
    if (key == kDictEmpty) {
      atomicOr(overflow, 1u);
      continue;
    }
    uint32_t h = dict_hash(key);
    bool done = false;
    for (int probe = 0; probe < kDictTable && !done; probe++) {
      const unsigned long long cur = ((volatile unsigned long long*)table)[h];
      if (cur == key) {
        done = true;
      } else if (cur == kDictEmpty) {
        const unsigned long long prev = atomicCAS(table + h, kDictEmpty, key);
        if (prev == kDictEmpty || prev == key) done = true;
        else h = (h + 1) & (kDictTable - 1);  // lost the race to another key: probe on
      } else {
        h = (h + 1) & (kDictTable - 1);
      }
    }
    if (!done) atomicOr(overflow, 1u);
  }
}

static __global__ void __launch_bounds__(kBlock) k_dict_pack(const int32_t* __restrict__ cols,
                                                      const double* __restrict__ vals, int64_t n,
                                                      const unsigned long long* __restrict__ table,
                                                      const uint8_t* __restrict__ tidx,
                                                      uint32_t* __restrict__ words) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const unsigned long long key = (unsigned long long)__double_as_longlong(vals[i]);
    uint32_t h = dict_hash(key);
    while (table[h] != key) h = (h + 1) & (kDictTable - 1);  // present by construction
    words[i] = (uint32_t)cols[i] | ((uint32_t)tidx[h] << kPackShift);
  }
}

// Complex H (the reference's complex(8) arithmetic, ED_SPARSE_MATRIX.f90:11-29):
// the same words over a dictionary of distinct (re, im) pairs.  Keys are a
// 64-bit mix of the two bit patterns; the inserting thread records the pair,
// and the pack kernel checks every slot's pair bit for bit against its entry
// (a hash collision between two pairs flags overflow: the plain arrays serve).
__device__ __forceinline__ unsigned long long pair_key(double2 v) {
  unsigned long long a = (unsigned long long)__double_as_longlong(v.x);
  unsigned long long b = (unsigned long long)__double_as_longlong(v.y);
  unsigned long long k = a ^ (b * 0x9E3779B97F4A7C15ull + 0x632BE59BD9B4E019ull + (a << 6) + (a >> 2));
  return k == kDictEmpty ? 0x7ff8dead00000001ull : k;
}

static __global__ void __launch_bounds__(kBlock) k_dict_insert_c(const double2* __restrict__ vals, int64_t n,
                                                          unsigned long long* table, double2* reps,
                                                          unsigned int* overflow) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const double2 v = vals[i];
    const unsigned long long key = pair_key(v);
    if (!wave_key_leader(key)) continue;  // (pairs with equal keys are checked at pack time)
    uint32_t h = dict_hash(key);
    bool done = false;
    for (int probe = 0; probe < kDictTable && !done; probe++) {
      const unsigned long long cur = ((volatile unsigned long long*)table)[h];
      if (cur == key) {
        done = true;
      } else if (cur == kDictEmpty) {
        const unsigned long long prev = atomicCAS(table + h, kDictEmpty, key);
        if (prev == kDictEmpty) {
          reps[h] = v;  // the inserting thread records the pair
          done = true;
        } else if (prev == key) {
          done = true;
        } else {
          h = (h + 1) & (kDictTable - 1);
        }
      } else {
        h = (h + 1) & (kDictTable - 1);
      }
    }
    if (!done) atomicOr(overflow, 1u);
  }
}

static __global__ void __launch_bounds__(kBlock) k_dict_pack_c(const int32_t* __restrict__ cols,
                                                        const double2* __restrict__ vals, int64_t n,
                                                        const unsigned long long* __restrict__ table,
                                                        const double2* __restrict__ reps,
                                                        const uint8_t* __restrict__ tidx,
                                                        uint32_t* __restrict__ words,
                                                        unsigned int* overflow) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    const double2 v = vals[i];
    const unsigned long long key = pair_key(v);
    uint32_t h = dict_hash(key);
    while (table[h] != key) h = (h + 1) & (kDictTable - 1);  // present by construction
    const double2 r = reps[h];
    if (__double_as_longlong(r.x) != __double_as_longlong(v.x) ||
        __double_as_longlong(r.y) != __double_as_longlong(v.y))
      atomicOr(overflow, 1u);
    words[i] = (uint32_t)cols[i] | ((uint32_t)tidx[h] << kPackShift);
  }
}

template <bool HC, bool VC, int NT, class Epi, int CH = kChunk>
__global__ void __launch_bounds__(kBlock) k_spmv_pk(const val_t<HC>* __restrict__ diag,
                                                    const int64_t* __restrict__ sptr,
                                                    const uint32_t* __restrict__ words,
                                                    const val_t<HC>* __restrict__ dict,
                                                    const val_t<VC>* __restrict__ x,
                                                    const val_t<VC>* __restrict__ xr, int64_t dim,
                                                    int64_t nslice, Epi epi, int xcd) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  if (epi.skip()) return;
  epi.prepare();
  double part = 0.0;
  // dictionary in LDS: its lookups leave the vector-memory pipe to the gathers
  __shared__ H sdict[256];
  sdict[threadIdx.x] = dict[threadIdx.x];  // kBlock == 256 == dictionary capacity
  __syncthreads();
  auto body = [&](int64_t i) {
    {
      // one slice per wavefront (kBlock is a multiple of 64 and lane 0 holds the
      // slice's first row): slice pointer and width are wave-uniform, so the
      // pointer loads and the k-loop bound live in scalar registers
      const int64_t s = (int64_t)__builtin_amdgcn_readfirstlane((int)(i >> 6));
      const int64_t s0 = sptr[s];
      const int w = (int)((sptr[s + 1] - s0) >> 6);
      const uint32_t* wp = words + s0 + (i & 63);
      const V xi = xr[i];
      const H dg = ldh<NT>(diag + i);
      // branch-free chunks: slots past the row width reload the last slot
      // (same lines, no new traffic) and are dropped by a select, so every
      // load of a chunk is issued before the first wait; the diagonal
      // product is formed after the first chunk's loads are in flight (the
      // sum order stays spMatVec_cc's: diagonal first)
      V acc;
      if (w == 0) {
        acc = add(vzero<V>(), mul(dg, xi));
      } else {
        const int wm = w - 1;
        for (int k0 = 0; k0 < w; k0 += CH) {
          uint32_t c[CH];
#pragma unroll
          for (int k = 0; k < CH; k++) c[k] = ldm<NT>(wp + 64 * min(k0 + k, wm));
          V g[CH];
          H h[CH];
#pragma unroll
          for (int k = 0; k < CH; k++) {
            g[k] = x[c[k] & kPackColMask];
            h[k] = sdict[c[k] >> kPackShift];
          }
          asm volatile("" ::: "memory");  // every gather in flight before the first use (complex: see k_spmv_sa)
          if (k0 == 0) acc = add(vzero<V>(), mul(dg, xi));
#pragma unroll
          for (int k = 0; k < CH; k++) acc = sel(k0 + k < w, add(acc, mul(h[k], g[k])), acc);
        }
      }
      part += epi.row(i, acc, xi);
    }
  };
  {
    // xcd: blocks are dealt round-robin to the 8 XCDs; remap so that each XCD
    // sweeps one contiguous range of rows (its L2 then serves the v gathers
    // shared by neighbouring rows)
    int64_t b = blockIdx.x;
    if (xcd) b = (b & 7) * (gridDim.x >> 3) + (b >> 3);
    for (int64_t i = b * kBlock + threadIdx.x; i < nslice * 64; i += (int64_t)gridDim.x * kBlock)
      if (i < dim) body(i);
  }
  epi.finish(part);
}

// ---------------------------------------------------- matrix-free (generic)
// directMatVec_cc (DIRECT_HxV.f90:21-92) in gather form, for every ed_mode.
// One wavefront per chunk of <= 64 consecutive rows of one idw block (the
// lanes share the down pattern idw and take consecutive up patterns of the
// block's class).  The row's elements come from the host-built op list of
// its block, in gen_row order (direct_candidates):
//   - UNI ops (terms acting on down levels only): condition, sign and target
//     block are the same for every lane, resolved on the host into a row
//     offset and a signed value — one coalesced gather, no per-lane work;
//   - LANE ops (terms touching up levels): condition, target pattern and
//     Jordan-Wigner sign per lane from the lane's up pattern (bit masks and
//     popc), target row off[idw'] (block-uniform, from the op) + rank of the
//     target up pattern (LDS table); the part of the sign that depends on
//     the block's down bits and the string's constant are folded into the
//     op's value on the host.
// The rank table (16-bit, 2^Ns entries) and the up patterns of every class
// (16-bit, 2^Ns) are staged in LDS once per workgroup; ops are read with
// scalar loads.  Ops go in groups of kDirGroup whose UNI/LANE pattern is a
// compile-time case (DirGroup::lanes selects one of 16 specialised bodies:
// no per-op scalar branch, a UNI op costs one address add and the product);
// every gather of a group is issued before the group is summed, in order,
// into the row: the same products and additions as k_spmv (a lane whose op
// does not fire gathers out of range, reads 0 and adds a zero product), so
// H·v equals the stored kernel's.  The diagonal is gen_row's own (gen_diag),
// evaluated once per sector by k_gen_diag into a vector (8 or 16 B per row).
// The two directions of a hop on up levels are one op (kDirXor, build_direct):
// ~half the per-lane evaluations of a normal-mode row.
// Round-4 counters (nonSU2 N26, an SQ_* pass of tools/spmv_probe.py): the kernel issued ~20
// VALU and ~22 SALU instructions per op (per-op kind branches, per-lane
// selects and sign assembly) and was issue-bound, not L1-bound.
constexpr int kDirBlock = 1024;
constexpr int kDirGroup = 4;
constexpr int kDirRows = 2;  // complex vectors: chunks of up to 64 * kDirRows rows (two per lane)
// Host form of one op (build_direct), before it is folded into a DirGroup:
//   fires  = (m & req_mask) == req_val && popc(m & xm) == (kind has kDirXor)
//   target = delta + rank[(m ^ flip) & up-mask]
//   sign   = (-1)^(popc(m & smask) + c0)
struct DirOp {
  uint32_t req_mask, req_val, flip, smask, xm;
  int32_t delta;
  int32_t kind;   // kDirLane | kDirC0 | kDirImSigned | kDirPad | kDirXor
  double re, im;  // before the sign
};
// kDirXor: merged hop pair, fires when exactly one of the two flip bits is set
constexpr int kDirLane = 1, kDirC0 = 2, kDirImSigned = 4, kDirPad = 8, kDirXor = 16;
// kDirGroup ops field by field in 64-byte lines (three s_load_dwordx16).
// Fields act on the lane's UP pattern u only (the block's down bits are
// resolved on the host):
//   LANE op j: fires = popc((u ^ cval) & cmask) == xv  (xv = 0: the up bits of
//              cmask equal cval; xv = 1: a merged hop pair, exactly one of its
//              two bits set)
//              target = delta + rank[u ^ flipu], value = (re, im) * (-1)^popc(u & smasku)
//              (the imaginary part signed only where bit j of imsig is set)
//   UNI op j:  target = delta + rank[u] (the lane's own rank), value (re, im)
//   pads:      UNI ops of value 0 on the row's own block
struct __align__(64) DirGroup {
  uint32_t cmask[kDirGroup], cval[kDirGroup], flipu[kDirGroup], smasku[kDirGroup];
  int32_t delta[kDirGroup];
  uint32_t xm[kDirGroup], xv[kDirGroup];  // xm: the merged pair's bits (host check only)
  uint32_t lanes, imsig, pad_[2];  // lanes: bit j = op j is a LANE op
  double re[kDirGroup], im[kDirGroup];
};
static_assert(sizeof(DirGroup) == 192, "DirGroup: three 64-byte scalar loads");
struct DirChunk {
  int32_t row;    // row of lane 0
  uint32_t idw;   // down pattern of the block
  int32_t pat0;   // index of lane 0's up pattern in the by-class table
  int32_t n;      // rows in the chunk (<= 64 R)
  int32_t op0, nop;  // the block's ops: [op0, op0 + nop), nop a multiple of kDirGroup
  int32_t pad[2];
};

// element gathers through a raw buffer resource: byte offsets in 32-bit
// unsigned arithmetic over a resource of exactly the vector's bytes, so the
// host admits k_direct only for vectors of < 2^32 bytes (kDirMaxVecBytes;
// launch_direct refuses larger ones); an offset at or past the end reads 0
constexpr uint64_t kDirMaxVecBytes = 0xffffffffull;
template <bool VC>
__device__ __forceinline__ val_t<VC> ld_rsrc_b(__amdgpu_buffer_rsrc_t r, uint32_t byte) {
  if constexpr (VC) {
    const auto q = __builtin_amdgcn_raw_buffer_load_b128(r, (int)byte, 0, 0);
    return __builtin_bit_cast(double2, q);
  } else {
    const auto q = __builtin_amdgcn_raw_buffer_load_b64(r, (int)byte, 0, 0);
    return __builtin_bit_cast(double, q);
  }
}

__device__ __forceinline__ double flip_sign(double v, uint32_t neg) {
  return __longlong_as_double(__double_as_longlong(v) ^ ((long long)neg << 63));
}

// Diagonal of every row of a matrix-free sector: gen_diag, the value the
// stored build puts in its diagonal slot (k_fill), so k_direct stays
// bit-identical to k_spmv.
template <bool HC>
__global__ void __launch_bounds__(kBlock) k_gen_diag(const EdModel* __restrict__ Mp,
                                                     const uint32_t* __restrict__ map, int64_t n,
                                                     val_t<HC>* __restrict__ out) {
  const EdModel& M = *Mp;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    double re, im;
    gen_diag(M, map[i], &re, &im);
    out[i] = mk<HC>(re, im);
  }
}

// One op group with UNI/LANE pattern M (bit j: op j is a LANE op), summed
// into the rows' accumulators in op order.  Every lane holds R rows (the
// group's scalar data serve both; R = 2: chunks of 128 rows).  ownb: a
// row's own rank in bytes; oobb: the byte offset past the vector (gathers
// there read 0).
template <int M, bool HC, bool VC, int R>
__device__ __forceinline__ void dir_group(const DirGroup& G, const uint32_t* up, const uint32_t* ownb, uint32_t oobb,
                                          const uint16_t* __restrict__ srank, __amdgpu_buffer_rsrc_t xr,
                                          val_t<VC>* acc) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  constexpr uint32_t lsz = VC ? 4u : 3u;
  // real H on real vectors: the lane's sign goes onto the gathered value
  // ((-g) h == g (-h) bit for bit), which keeps h a scalar operand
  constexpr bool GSIGN = !HC && !VC;
  uint32_t rk[R][kDirGroup];
#pragma unroll
  for (int j = 0; j < kDirGroup; j++)
    if ((M >> j) & 1) {
#pragma unroll
      for (int r = 0; r < R; r++) rk[r][j] = srank[up[r] ^ G.flipu[j]];
    }
  uint32_t off[R][kDirGroup], neg[R][kDirGroup];
  H h[R][kDirGroup];
#pragma unroll
  for (int j = 0; j < kDirGroup; j++) {
    const uint32_t base = (uint32_t)G.delta[j] << lsz;  // scalar
#pragma unroll
    for (int r = 0; r < R; r++) {
      neg[r][j] = 0;
      if ((M >> j) & 1) {
        // condition: popc((u ^ cval) & cmask) == xv (xv = 1: a merged hop
        // pair, exactly one of its two bits set; 0: the bits equal cval)
        const bool f = (uint32_t)__builtin_popcount((up[r] ^ G.cval[j]) & G.cmask[j]) == G.xv[j];
        neg[r][j] = (uint32_t)__builtin_popcount(up[r] & G.smasku[j]) & 1u;
        off[r][j] = f ? base + (rk[r][j] << lsz) : oobb;
        if constexpr (HC)
          h[r][j] = make_double2(flip_sign(G.re[j], neg[r][j]),
                                 ((G.imsig >> j) & 1u) ? flip_sign(G.im[j], neg[r][j]) : G.im[j]);
        else if constexpr (GSIGN)
          h[r][j] = G.re[j];
        else
          h[r][j] = flip_sign(G.re[j], neg[r][j]);
      } else {
        off[r][j] = base + ownb[r];
        h[r][j] = mk<HC>(G.re[j], G.im[j]);
      }
    }
  }
  V g[R][kDirGroup];
#pragma unroll
  for (int j = 0; j < kDirGroup; j++)
#pragma unroll
    for (int r = 0; r < R; r++) g[r][j] = ld_rsrc_b<VC>(xr, off[r][j]);
#pragma unroll
  for (int j = 0; j < kDirGroup; j++)
#pragma unroll
    for (int r = 0; r < R; r++) {
      if constexpr (GSIGN) {
        if ((M >> j) & 1) g[r][j] = flip_sign(g[r][j], neg[r][j]);
      }
      acc[r] = add(acc[r], mul(h[r][j], g[r][j]));
    }
}

// R: rows per lane (chunks of up to 64 R rows; one pass over the ops serves
// the R rows, their scalar data shared).  Real vectors R = 1: nonSU2 N26
// 0.279 against 0.292 ms with R = 2; complex vectors R = 2: 0.378 against
// 0.435 ms.  The host keeps a chunk list for each.
template <bool HC, bool VC, bool PATLDS, int R, class Epi>
__global__ void __launch_bounds__(kDirBlock) k_direct(const val_t<HC>* __restrict__ ddiag,
                                                      const DirChunk* __restrict__ chunks, int nchunk,
                                                      const DirGroup* __restrict__ grp,
                                                      const uint16_t* __restrict__ rank_g,
                                                      const uint16_t* __restrict__ pat_g,
                                                      const uint32_t* __restrict__ map, int ns,
                                                      const val_t<VC>* __restrict__ x, int64_t xdim, int64_t row0,
                                                      Epi epi) {
  using V = val_t<VC>;
  if (epi.skip()) return;
  epi.prepare();
  extern __shared__ __align__(16) unsigned char smem[];
  uint16_t* srank = (uint16_t*)smem;
  uint16_t* spat = srank + (1 << ns);
  if (ns >= 3) {  // 16-byte staging of the tables
    const int h = (1 << ns) / 8;
    const int n4 = (PATLDS ? 2 : 1) * h;
    const uint4* src0 = (const uint4*)rank_g;
    const uint4* src1 = (const uint4*)pat_g;
    for (int q = threadIdx.x; q < n4; q += kDirBlock) ((uint4*)smem)[q] = q < h ? src0[q] : src1[q - h];
  } else {
    for (int q = threadIdx.x; q < (1 << ns); q += kDirBlock) {
      srank[q] = rank_g[q];
      if (PATLDS) spat[q] = pat_g[q];
    }
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // chunk data and ops: scalar loads
  const uint32_t mask = (1u << ns) - 1u;
  constexpr uint32_t lsz = VC ? 4u : 3u;
  // chunk schedule: with a grid of 8k blocks each XCD (blocks b = x mod 8)
  // walks one contiguous eighth of the chunks, so its L2 serves the gathers
  // neighbouring rows share
  int c, cend, cstep;
  if ((gridDim.x & 7) == 0) {
    const int xcd = blockIdx.x & 7;
    c = (int)((int64_t)nchunk * xcd / 8) + (int)(blockIdx.x >> 3) * (kDirBlock / 64) + wv;
    cend = (int)((int64_t)nchunk * (xcd + 1) / 8);
    cstep = (int)(gridDim.x >> 3) * (kDirBlock / 64);
  } else {
    c = blockIdx.x * (kDirBlock / 64) + wv;
    cend = nchunk;
    cstep = gridDim.x * (kDirBlock / 64);
  }
  // the resource spans exactly the sector vector: offset oobb reads 0
  const uint32_t oobb = (uint32_t)((uint64_t)xdim * sizeof(V));
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc((void*)x, (short)0, (int)oobb, 0x00020000);
  double part = 0.0;
  for (; c < cend; c += cstep) {
    const DirChunk ch = chunks[c];  // up to 64 R rows; lane holds rows ch.row + 64 r + lane
    uint32_t up[R], ownb[R];
    int row[R];
    bool on[R];
    V xi[R], acc[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int l = lane + 64 * r;
      on[r] = l < ch.n;
      row[r] = ch.row + (on[r] ? l : 0);
      if constexpr (PATLDS) up[r] = spat[ch.pat0 + (on[r] ? l : 0)];
      else up[r] = map[row[r]] & mask;
      ownb[r] = (uint32_t)srank[up[r]] << lsz;
      xi[r] = x[row[r]];
      acc[r] = add(vzero<V>(), mul(ddiag[row[r] - row0], xi[r]));
    }
    const int g1 = (ch.op0 + ch.nop) / kDirGroup;
    for (int gi = ch.op0 / kDirGroup; gi < g1; gi++) {
      const DirGroup G = grp[gi];
      switch (G.lanes) {  // scalar: one uniform jump per group
#define ED_DIRG(M) \
  case M: dir_group<M, HC, VC, R>(G, up, ownb, oobb, srank, xr, acc); break;
        ED_DIRG(0) ED_DIRG(1) ED_DIRG(2) ED_DIRG(3) ED_DIRG(4) ED_DIRG(5) ED_DIRG(6) ED_DIRG(7)
        ED_DIRG(8) ED_DIRG(9) ED_DIRG(10) ED_DIRG(11) ED_DIRG(12) ED_DIRG(13) ED_DIRG(14)
        default: dir_group<15, HC, VC, R>(G, up, ownb, oobb, srank, xr, acc); break;
#undef ED_DIRG
      }
    }
#pragma unroll
    for (int r = 0; r < R; r++)
      if (on[r]) part += epi.row((int64_t)row[r] - row0, acc[r], xi[r]);
  }
  epi.template finish<kDirBlock>(part);
}

// ------------------------------------------- matrix-free (Kronecker form)
// Normal mode without spin-exchange/pair-hopping: every off-diagonal term
// moves one spin species only, and the Jordan-Wigner string of a down-spin
// hop crosses all up bits twice (sign cancels).  With v viewed as the
// DimDw x DimUp matrix V (row = rank(idw), column = rank(iup), exactly the
// reference order), H v = D.V + V Hup^T + Hdw V.  Hup/Hdw are tiny ELL
// tables (column-major [k][row]), D = Aup[iu] + Adw[iw] + U[imp(iu)][imp(iw)].
template <bool HC>
struct KronArgs {
  using H = val_t<HC>;
  int64_t dimup, dimdw;
  int degup, degdw, nimp;
  const int32_t* upc;
  const H* upv;
  const int32_t* dwc;
  const H* dwv;
  const H* aup;
  const H* adw;
  const double* uimp;    // [nimp*nimp]
  const uint8_t* impu;   // [dimup]
  const uint8_t* impd;   // [dimdw]
};

template <bool HC, bool VC, class Epi>
__global__ void __launch_bounds__(kBlock) k_kron(KronArgs<HC> K, const val_t<VC>* __restrict__ x,
                                                 int64_t dim, int64_t nslice, Epi epi) {
  using V = val_t<VC>;
  if (epi.skip()) return;
  epi.prepare();
  double part = 0.0;
  const int64_t du = K.dimup;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < nslice * 64;
       i += (int64_t)gridDim.x * kBlock) {
    if (i < dim) {
      const int64_t iw = i / du;
      const int64_t iu = i - iw * du;
      const V xi = x[i];
      auto d = add(add(K.aup[iu], K.adw[iw]), mk<HC>(K.uimp[K.impu[iu] * K.nimp + K.impd[iw]], 0.0));
      V acc = mul(d, xi);
      const V* xrow = x + iw * du;
      for (int k = 0; k < K.degup; k++) {
        const int64_t q = (int64_t)k * du + iu;
        acc = add(acc, mul(K.upv[q], xrow[K.upc[q]]));
      }
      for (int k = 0; k < K.degdw; k++) {
        const int64_t q = (int64_t)k * K.dimdw + iw;
        acc = add(acc, mul(K.dwv[q], x[(int64_t)K.dwc[q] * du + iu]));
      }
      part += epi.row(i, acc, xi);
    }
  }
  epi.finish(part);
}

// ------------------------------- matrix-free Kronecker form, two passes
// k_kron reads every V row ~(1 + degdw) times: its down-hop gathers of the
// rows V[iw'][:] have no cache locality (a hop jumps far in rank) and come
// from the Infinity Cache, and its up-hop gathers and table loads go through
// L1/L2 one thread per row (N28: 0.91 GB fetched for 0.19 GB of v/Hv).  Here
// the two index directions are split so that each pass has locality:
//   pass U (k_kron_up)  y[iw][:] = D[iw][:] .* V[iw][:] + V[iw][:] Hup^T
//     one 1024-thread workgroup per 2 rows (1 if LDS is short) at a time:
//     the rows are staged in LDS (two sets, one barrier per step), the
//     up-hop gathers are LDS
//     reads, the thread's up-hop words {col:16 | value index:8} and diagonal
//     factors sit in registers for all rows of the workgroup;
//   pass D (k_kron_dw)  Hv[iw][c] = y[iw][c] + sum_k Hdw[iw][k] V[k'][c]
//     one wavefront per (row, 64-column chunk); each XCD sweeps its own
//     column chunks, all its workgroups on the same chunk at once, so the
//     chunk V[:][c0:c0+64] (dimdw x 512 B, 1.8 MB at N28) stays in the XCD's
//     4 MB L2 and every V element is fetched once; the down-hop words are
//     wave-uniform (scalar loads), values from an LDS dictionary, and all
//     loads of a wave's 4 rows are issued before the first use.
// Term order per element = k_kron's (diagonal, up hops in slot order, down
// hops in slot order): bit-identical results.  The epilogue runs in pass D;
// pass U writes into the epilogue's scratch (its output buffer).
constexpr int kKronUpBlock = 1024;
constexpr int kKronDictMax = 256;
constexpr int kKronRowsPerWave = 4;   // pass D tile: 4 waves x 4 rows x 64 columns
constexpr int kKronUimpMax = 64;      // U[imp][imp] table entries (Norb <= 3)
// steps of staged rows prefetched in registers (2 and 3 measured slower:
// register pressure)
constexpr int kKronUpPF = 1;

template <bool HC, bool VC, int CPT, int DEG, int kKronUpRows>
__global__ void __launch_bounds__(kKronUpBlock) k_kron_up(KronArgs<HC> K, const uint32_t* __restrict__ upw,
                                                          const val_t<HC>* __restrict__ updict, int ndict,
                                                          const val_t<VC>* __restrict__ x, val_t<VC>* y) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  extern __shared__ __align__(16) unsigned char smem[];
  H* sdict = (H*)smem;
  // the impurity interaction table U[imp(iu)][imp(iw)] (<= 8 x 8) in LDS: a
  // global load there sat in every step's dependency chain (L2 round trip
  // between the barrier and the first FMA, exposed at one workgroup per CU)
  double* suimp = (double*)(smem + kKronDictMax * sizeof(H));
  const int du = (int)K.dimup;
  const int64_t dd = K.dimdw;
  const int dup = (du + 1) & ~1;
  V* bufs = (V*)(smem + kKronDictMax * sizeof(H) + kKronUimpMax * sizeof(double));  // 2 sets x kKronUpRows rows
  const int t = threadIdx.x;
  const int64_t G = gridDim.x;
  for (int q = t; q < ndict; q += kKronUpBlock) sdict[q] = updict[q];
  for (int q = t; q < K.nimp * K.nimp; q += kKronUpBlock) suimp[q] = K.uimp[q];
  const int degup = K.degup;
  uint32_t w[CPT][DEG];
  H au[CPT];
  int imu[CPT];
#pragma unroll
  for (int j = 0; j < CPT; j++) {
    const int iu = t + kKronUpBlock * j;
    const bool ok = iu < du;
#pragma unroll
    for (int k = 0; k < DEG; k++) w[j][k] = (ok && k < degup) ? upw[(int64_t)k * du + iu] : 0u;
    au[j] = ok ? K.aup[iu] : mk<HC>(0.0, 0.0);
    imu[j] = ok ? (int)K.impu[iu] : 0;
  }
  // kKronUpRows rows per step (iw = base + r*G), the next step's rows
  // prefetched into registers while this step's are computed; with 2 rows
  // the LDS image is interleaved ([column][row]): one gather fetches the
  // column of both rows (ds_read_b128 for real vectors)
  struct Pair {
    V a, b;
  };
  // kKronUpPF steps of rows in flight in registers
  V xr[kKronUpPF][kKronUpRows][CPT];
  int64_t base = blockIdx.x;
#pragma unroll
  for (int f = 0; f < kKronUpPF; f++)
#pragma unroll
    for (int r = 0; r < kKronUpRows; r++)
#pragma unroll
      for (int j = 0; j < CPT; j++) {
        const int iu = t + kKronUpBlock * j;
        const int64_t iw = base + (f * kKronUpRows + r) * G;
        xr[f][r][j] = (iw < dd && iu < du) ? x[(int)iw * du + iu] : vzero<V>();
      }
  // down-spin diagonal factors of the rows in flight (wave-uniform), loaded
  // with them
  H adn[kKronUpPF][kKronUpRows];
  int imdn[kKronUpPF][kKronUpRows];
#pragma unroll
  for (int f = 0; f < kKronUpPF; f++)
#pragma unroll
    for (int r = 0; r < kKronUpRows; r++) {
      const int64_t iw = base + (f * kKronUpRows + r) * G;
      const int64_t iwc = iw < dd ? iw : 0;
      adn[f][r] = K.adw[iwc];
      imdn[f][r] = K.impd[iwc];
    }
  int pb = 0;
  for (; base < dd; base += kKronUpRows * G) {
    V* buf = bufs + (size_t)pb * kKronUpRows * dup;
#pragma unroll
    for (int j = 0; j < CPT; j++) {
      const int iu = t + kKronUpBlock * j;
      if (iu < du) {
        if constexpr (kKronUpRows == 2) ((Pair*)buf)[iu] = Pair{xr[0][0][j], xr[0][1][j]};
        else buf[iu] = xr[0][0][j];
      }
    }
    __syncthreads();  // rows staged; (two sets: the reads of the step before last are done)
    H ad[kKronUpRows];
    int imd[kKronUpRows];
#pragma unroll
    for (int r = 0; r < kKronUpRows; r++) {
      ad[r] = adn[0][r];
      imd[r] = imdn[0][r];
    }
#pragma unroll
    for (int f = 0; f + 1 < kKronUpPF; f++)
#pragma unroll
      for (int r = 0; r < kKronUpRows; r++) {
        adn[f][r] = adn[f + 1][r];
        imdn[f][r] = imdn[f + 1][r];
#pragma unroll
        for (int j = 0; j < CPT; j++) xr[f][r][j] = xr[f + 1][r][j];
      }
    const int64_t nb = base + kKronUpPF * kKronUpRows * G;
#pragma unroll
    for (int r = 0; r < kKronUpRows; r++) {
      const int64_t iw = nb + r * G;
      const int64_t iwc = iw < dd ? iw : 0;
      adn[kKronUpPF - 1][r] = K.adw[iwc];
      imdn[kKronUpPF - 1][r] = K.impd[iwc];
#pragma unroll
      for (int j = 0; j < CPT; j++) {
        const int iu = t + kKronUpBlock * j;
        xr[kKronUpPF - 1][r][j] = (iw < dd && iu < du) ? x[(int)iw * du + iu] : vzero<V>();
      }
    }
    const bool second = kKronUpRows == 2 && base + G < dd;
#pragma unroll
    for (int j = 0; j < CPT; j++) {
      const int iu = t + kKronUpBlock * j;
      if (iu < du) {
        // the element's own value for the diagonal term is read back from the
        // staged row (no register copy: the prefetch ring needs the VGPRs)
        V xo[kKronUpRows];
        if constexpr (kKronUpRows == 2) {
          const Pair p = ((const Pair*)buf)[iu];
          xo[0] = p.a;
          xo[kKronUpRows - 1] = p.b;
        } else {
          xo[0] = buf[iu];
        }
        V acc[kKronUpRows];
#pragma unroll
        for (int r = 0; r < kKronUpRows; r++) {
          const auto d = add(add(au[j], ad[r]), mk<HC>(suimp[imu[j] * K.nimp + imd[r]], 0.0));
          acc[r] = mul(d, xo[r]);
        }
#pragma unroll
        for (int k = 0; k < DEG; k++)
          if (k < degup) {
            const H h = sdict[w[j][k] >> 16];
            const int col = w[j][k] & 0xffffu;
            if constexpr (kKronUpRows == 2) {
              const Pair p = ((const Pair*)buf)[col];
              acc[0] = add(acc[0], mul(h, p.a));
              acc[1] = add(acc[1], mul(h, p.b));
            } else {
              acc[0] = add(acc[0], mul(h, buf[col]));
            }
          }
        y[(int)base * du + iu] = acc[0];
        if (second) y[(int)(base + G) * du + iu] = acc[kKronUpRows - 1];
      }
    }
    pb ^= 1;
  }
}

// dwo[iw*DEG + k] = row index iw' of the k-th down-hop target row (its
// element offset is iw' * ld: ld = DimUp for the whole sector, nu for the
// DimDw x nu column strip of the within-sector split),
// dwi[iw*DEG + k] = its value's dictionary index (DEG slots per row, padded):
// one wave-uniform row is one s_load_dwordx8/x16 + one of the index bytes
// CW = 2 (real vectors, even ld and ncols, 16-byte aligned x and ypart): two
// adjacent columns per lane, 128 per wave — one 16-byte gather per hop
// instead of two 8-byte ones; the same per-element term order
template <bool HC, bool VC, int DEG, class Epi, int CW = 1>
__global__ void __launch_bounds__(kBlock) k_kron_dw(KronArgs<HC> K, const uint32_t* __restrict__ dwo,
                                                    const uint8_t* __restrict__ dwi,
                                                    const val_t<HC>* __restrict__ dwdict, int ndict,
                                                    const val_t<VC>* __restrict__ x, const val_t<VC>* ypart,
                                                    Epi epi, int ld, int ncols) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  if (epi.skip()) return;
  epi.prepare();
  __shared__ H sdict[kKronDictMax];
  for (int q = threadIdx.x; q < ndict; q += kBlock) sdict[q] = dwdict[q];
  __syncthreads();
  // 32-bit index arithmetic throughout (dim < 2^31, checked on the host): the
  // tile walk is scalar code, and 64-bit divisions there made the kernel
  // SALU-bound (29 M scalar instructions per launch at N28)
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  // rows of length ld, columns [0, ncols): the whole DimDw x DimUp view
  // (ld = ncols = DimUp) or a column strip; ypart == nullptr: no first-pass
  // part (the strip's down-hop sum alone)
  static_assert(CW == 1 || (CW == 2 && !VC), "two columns per lane: real vectors only");
  const int du = ld, dd = (int)K.dimdw;
  constexpr int CWID = 64 * CW;  // columns per chunk
  const int nchunk = (ncols + CWID - 1) / CWID;
  // rows per wave: 4 at <= 8 slots; 2 above (the R x DEG gathered values sit
  // in VGPRs: 4 x 16 doubles held 149 VGPRs, 3 waves/SIMD, scalar spills);
  // half that for complex vectors (4 x 8 complex: 157 VGPRs, 3 waves/SIMD)
  // and for two columns per lane
  // (4 rows per wave with two columns: 157 VGPRs, 3 waves/SIMD, slower)
  constexpr int R = (VC || CW == 2) ? (DEG <= 8 ? 2 : 1) : (DEG <= 8 ? kKronRowsPerWave : 2);
  constexpr int kTileRows = (kBlock / 64) * R;
  const int nrb = (dd + kTileRows - 1) / kTileRows;
  // blocks are dealt round-robin to the 8 XCDs: XCD x = blockIdx % 8 takes
  // the tiles [T x / 8, T (x + 1) / 8) of the chunk-major (chunk, row block)
  // order (T tiles), and its blocks walk them in order — every XCD the same
  // work, a chunk shared by at most two XCDs.  (Whole chunks dealt round-robin
  // left N28's 27 chunks as 4 on three XCDs and 3 on five: the pass took the
  // time of 4 chunks where the average is 3.4.)
  const int xcd = blockIdx.x & 7;
  const int g8 = gridDim.x >> 3;
  const int64_t T = (int64_t)nchunk * nrb;
  const int t1 = (int)(T * (xcd + 1) / 8);
  int t = (int)(T * xcd / 8) + (int)(blockIdx.x >> 3);
  int ch = t / nrb, rb = t - ch * nrb;
  double part = 0.0;
  for (; t < t1;) {
    const int iu = ch * CWID + lane * CW;
    const bool ok = iu < ncols;
    const int r0 = rb * kTileRows + wv * R;  // wave-uniform
    // every load of the wave's R rows in flight before any use
    uint32_t wo[R][DEG];
    uint8_t wi[R][DEG];
    int nk[R];  // the row's hop count (slot 0's top byte; trailing slots are padding)
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int rr = r0 + r < dd ? r0 + r : r0;
#pragma unroll
      for (int k = 0; k < DEG; k++) {
        const uint32_t wd = dwo[rr * DEG + k];
        if (k == 0) nk[r] = r0 + r < dd ? (int)(wd >> 24) : 0;
        wo[r][k] = (wd & 0xffffffu) * (uint32_t)du;
        wi[r][k] = dwi[rr * DEG + k];
      }
    }
    if constexpr (CW == 2) {
      typedef double d2 __attribute__((ext_vector_type(2)));
      const d2 z2 = {0.0, 0.0};
      d2 g[R][DEG], yv[R], xv[R];
#pragma unroll
      for (int r = 0; r < R; r++) {
        const int i = (r0 + r) * du + iu;
        const bool on = ok && r0 + r < dd;
#pragma unroll
        for (int k = 0; k < DEG; k++) {
          g[r][k] = z2;
          if (k < nk[r]) g[r][k] = on ? *(const d2*)(x + (int)wo[r][k] + iu) : z2;
        }
        xv[r] = on ? *(const d2*)(x + i) : z2;
        yv[r] = (on && ypart) ? *(const d2*)(ypart + i) : z2;  // (non-temporal: slower)
      }
#pragma unroll
      for (int r = 0; r < R; r++) {
        if (!ok || r0 + r >= dd) continue;
        double a0 = yv[r].x, a1 = yv[r].y;
#pragma unroll
        for (int k = 0; k < DEG; k++)
          if (k < nk[r]) {
            const H h = sdict[wi[r][k]];
            a0 = add(a0, mul(h, g[r][k].x));
            a1 = add(a1, mul(h, g[r][k].y));
          }
        const int i = (r0 + r) * du + iu;
        // the plain store epilogue writes Hv non-temporally (as EpiStore::row):
        // fewer of the chunk's V lines evicted by the Hv stream (N28 pass D
        // FETCH 275 -> 257 MB, H·v -1.5 %); one 16-byte store here
        if constexpr (std::is_same_v<Epi, EpiStore<VC>>) {
          __builtin_nontemporal_store(d2{a0, a1}, (d2*)(epi.hv + i));
        } else {
          part += epi.row((int64_t)i, a0, xv[r].x);
          part += epi.row((int64_t)i + 1, a1, xv[r].y);
        }
      }
      t += g8;
      rb += g8;
      while (rb >= nrb) {
        rb -= nrb;
        ch++;
      }
      continue;
    }
    V g[R][DEG], yv[R], xv[R];
#pragma unroll
    for (int r = 0; r < R; r++) {
      const int i = (r0 + r) * du + iu;
      const bool on = ok && r0 + r < dd;
#pragma unroll
      for (int k = 0; k < DEG; k++) {
        g[r][k] = vzero<V>();
        if (k < nk[r])  // wave-uniform: padding slots issue no gather
          g[r][k] = on ? x[(int)wo[r][k] + iu] : vzero<V>();
      }
      xv[r] = on ? x[i] : vzero<V>();
      yv[r] = (on && ypart) ? ypart[i] : vzero<V>();
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
      if (!ok || r0 + r >= dd) continue;
      V acc = yv[r];
#pragma unroll
      for (int k = 0; k < DEG; k++)
        if (k < nk[r]) acc = add(acc, mul(sdict[wi[r][k]], g[r][k]));
      part += epi.row((int64_t)((r0 + r) * du + iu), acc, xv[r]);
    }
    t += g8;
    rb += g8;
    while (rb >= nrb) {
      rb -= nrb;
      ch++;
    }
  }
  epi.finish(part);
}

// ------------------------------------ within-sector split
// H = D + Hup(x)1 + 1(x)Hdw on the DimDw x DimUp view.  A rank owning down
// rows [w0, w0+nw) applies the diagonal and the up-spin hops locally
// (k_kron_rows on its nw x DimUp block); the down-spin hops act along the
// other index and run on the DimDw x nu column strip it receives by an
// all-to-all (k_kron_cols).  Term order per element: diagonal,
// up hops | down hops — the two partial sums are added by the caller.
template <bool HC, bool VC>
__global__ void __launch_bounds__(kBlock) k_kron_rows(KronArgs<HC> K, int64_t w0, int64_t nw,
                                                      const val_t<VC>* __restrict__ x,
                                                      val_t<VC>* __restrict__ y) {
  using V = val_t<VC>;
  const int64_t du = K.dimup;
  for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < nw * du;
       q += (int64_t)gridDim.x * kBlock) {
    const int64_t r = q / du, iu = q - r * du, iw = w0 + r;
    auto d = add(add(K.aup[iu], K.adw[iw]), mk<HC>(K.uimp[K.impu[iu] * K.nimp + K.impd[iw]], 0.0));
    V acc = mul(d, x[q]);
    const V* xrow = x + r * du;
    for (int k = 0; k < K.degup; k++) {
      const int64_t t = (int64_t)k * du + iu;
      acc = add(acc, mul(K.upv[t], xrow[K.upc[t]]));
    }
    y[q] = acc;
  }
}

// z, yz: DimDw x nu row-major (down row iw, up column c fastest): exactly
// the concatenation of the row blocks an all-to-all delivers, so neither
// side of the exchange needs a transpose and the gathers z[iw'][c] are
// coalesced over c.
template <bool HC, bool VC>
__global__ void __launch_bounds__(kBlock) k_kron_cols(KronArgs<HC> K, int64_t nu,
                                                      const val_t<VC>* __restrict__ z,
                                                      val_t<VC>* __restrict__ yz, int accumulate) {
  using V = val_t<VC>;
  const int64_t dd = K.dimdw;
  for (int64_t q = (int64_t)blockIdx.x * kBlock + threadIdx.x; q < nu * dd;
       q += (int64_t)gridDim.x * kBlock) {
    const int64_t iw = q / nu, c = q - iw * nu;
    V acc = accumulate ? yz[q] : vzero<V>();
    for (int k = 0; k < K.degdw; k++) {
      const int64_t t = (int64_t)k * dd + iw;
      acc = add(acc, mul(K.dwv[t], z[(int64_t)K.dwc[t] * nu + c]));
    }
    yz[q] = acc;
  }
}

// -------------------------------- row split: columns the held rows gather
// One bit per sector column, set for every column an off-diagonal element of
// rows [row0, row0 + n) refers to (gen_row's elements: stored and matrix-free
// alike).  The halo of a rank's row block for the split H·v (edgpu.dist).
struct MarkAcc {
  DevIndex idx;
  uint32_t* mask;
  __device__ __forceinline__ void diag(double, double) {}
  __device__ __forceinline__ void off(uint32_t k, double, double) {
    const uint32_t c = (uint32_t)idx(k);
    atomicOr(mask + (c >> 5), 1u << (c & 31));
  }
};
static __global__ void __launch_bounds__(kBlock) k_mark_cols(const EdModel* __restrict__ Mp,
                                                      const uint32_t* __restrict__ map, int64_t n,
                                                      DevIndex idx, uint32_t* mask) {
  const EdModel& M = *Mp;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    MarkAcc a{idx, mask};
    gen_row(M, map[i], a);
  }
}

// ------------------------------------------------ GF seeds: c / c^+ |state>
// One thread per source row; every target row is hit at most once (the
// operator is injective on the Fock basis), so plain stores suffice.
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_apply_op(const uint32_t* __restrict__ map_src,
                                                     int64_t dim_src, DevIndex idx_dst, int op,
                                                     int level, const val_t<VC>* __restrict__ x,
                                                     val_t<VC>* __restrict__ y) {
  for (int64_t m = (int64_t)blockIdx.x * kBlock + threadIdx.x; m < dim_src;
       m += (int64_t)gridDim.x * kBlock) {
    const uint32_t st = map_src[m];
    const int occ = bit(st, level);
    if ((op == 1 && occ == 0) || (op == 0 && occ == 1)) {
      const double sg = jw_sign(st, level);
      const uint32_t t = st ^ (1u << level);
      y[idx_dst(t)] = scl(sg, x[m]);
    }
  }
}

template <bool VC>
__global__ void __launch_bounds__(kBlock) k_apply_op_acc(const uint32_t* __restrict__ map_src,
                                                         int64_t dim_src, DevIndex idx_dst, int op,
                                                         int level, double cr, double ci,
                                                         const val_t<VC>* __restrict__ x,
                                                         val_t<VC>* __restrict__ y) {
  for (int64_t m = (int64_t)blockIdx.x * kBlock + threadIdx.x; m < dim_src;
       m += (int64_t)gridDim.x * kBlock) {
    const uint32_t st = map_src[m];
    const int occ = bit(st, level);
    if ((op == 1 && occ == 0) || (op == 0 && occ == 1)) {
      const double sg = jw_sign(st, level);
      const int32_t j = idx_dst(st ^ (1u << level));
      if constexpr (VC) {
        const double2 v = x[m];
        const double2 t = make_double2(sg * (cr * v.x - ci * v.y), sg * (cr * v.y + ci * v.x));
        y[j] = make_double2(y[j].x + t.x, y[j].y + t.y);
      } else {
        y[j] = y[j] + cr * (sg * x[m]);
      }
    }
  }
}

// ------------------------------------------------ GF pole sums (device G)
// add_to_lanczos_gf_normal (ED_GF_NORMAL.f90:620-631) / _nonsu2
// (ED_GF_NONSU2.f90:936-950): for every frequency i, fraction by fraction in
// list order and pole by pole (j ascending), exactly the reference's sequence
// of additions into G(i):
//   G(i) = G(i) + peso_j / (iw_i - isign*de_j),  de_j = E_j - Ei,
//   peso_j = (pesoBZ * z_j) * z_j,  iw = (0, wm_i) or (wr_i, eps).
// One thread per frequency (Matsubara then real axis); the fraction and pole
// data are wave-uniform (scalar loads); G stays in HBM across seeds.
struct GfFrac {
  int32_t p0, np, comp, isign;
  double pr, pi, ei;  // pesoBZ (complex), Ei
  double pad;
};

// Smith's complex division (the scaling gfortran/flang use for complex /)
__device__ __forceinline__ double2 cdiv(double2 p, double a, double b) {
  if (fabs(b) <= fabs(a)) {
    const double r = b / a, den = a + b * r;
    return make_double2((p.x + p.y * r) / den, (p.y - p.x * r) / den);
  }
  const double r = a / b, den = a * r + b;
  return make_double2((p.x * r + p.y) / den, (p.y * r - p.x) / den);
}

static __global__ void __launch_bounds__(kBlock) k_gf_poles(const GfFrac* __restrict__ fr, int nfrac,
                                                     const double* __restrict__ E, const double* __restrict__ z,
                                                     const double* __restrict__ wm, int lmats,
                                                     const double* __restrict__ wr, int lreal, double eps,
                                                     double2* __restrict__ gm, double2* __restrict__ gr) {
  const int t = blockIdx.x * kBlock + threadIdx.x;
  if (t >= lmats + lreal) return;
  const bool mats = t < lmats;
  const int i = mats ? t : t - lmats;
  const double re_w = mats ? 0.0 : wr[i];   // iw = xi*wm(i) = (0, wm); dcmplx(wr(i), eps)
  const double im_w = mats ? wm[i] : eps;
  double2* G = mats ? gm : gr;
  const int L = mats ? lmats : lreal;
  int cur = -1;
  double2 g = make_double2(0.0, 0.0);
  for (int f = 0; f < nfrac; f++) {
    const GfFrac q = fr[f];
    if (q.comp != cur) {
      if (cur >= 0) G[(int64_t)cur * L + i] = g;
      cur = q.comp;
      g = G[(int64_t)cur * L + i];
    }
    const double sgn = (double)q.isign;
    for (int j = 0; j < q.np; j++) {
      const double zj = z[q.p0 + j];
      const double de = E[q.p0 + j] - q.ei;
      const double2 peso = make_double2((q.pr * zj) * zj, (q.pi * zj) * zj);
      const double d = sgn * de;
      const double2 c = cdiv(peso, re_w - d, im_w);
      g = make_double2(g.x + c.x, g.y + c.y);
    }
  }
  if (cur >= 0) G[(int64_t)cur * L + i] = g;
}

// ------------------------------------------------------------ Lanczos misc
// Start: R holds v0.  P <- 0; b_1 = ||R|| -> st.  (iteration 1 normalises, :96-101)
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_lanc_init(const val_t<VC>* __restrict__ R,
                                                      val_t<VC>* __restrict__ P, int64_t dim,
                                                      LancState* st, double thresh,
                                                      RedSlot slot) {
  using V = val_t<VC>;
  double part = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim;
       i += (int64_t)gridDim.x * kBlock) {
    V r = R[i];
    part += redot(r, r);
    P[i] = vzero<V>();
  }
  double tot;
  if (grid_reduce_last(part, slot, &tot) && threadIdx.x == 0) {
    double b = sqrt(tot);
    st->beta = b;
    st->invb = 1.0 / b;
    st->alpha = 0.0;
    st->thresh = thresh;
    st->iter = 0;
    st->done = (b == 0.0) ? 1 : 0;
  }
}

// Lanczos step, part B: w = W - alpha*v (v = P), R <- w, b = ||w||.  (:111-113)
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_lanc_b(const val_t<VC>* __restrict__ W,
                                                   const val_t<VC>* __restrict__ P,
                                                   val_t<VC>* __restrict__ R, int64_t dim,
                                                   LancState* st, double* beta_out,
                                                   RedSlot slot) {
  using V = val_t<VC>;
  if (st->done) return;
  const double a = st->alpha;
  double part = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim;
       i += (int64_t)gridDim.x * kBlock) {
    V w = sub(W[i], scl(a, P[i]));
    R[i] = w;
    part += redot(w, w);
  }
  if (!slot.counter) {
    block_partial(part, slot.partials);
    return;
  }
  double tot;
  if (grid_reduce_last(part, slot, &tot) && threadIdx.x == 0) lanc_set_beta(tot, st, beta_out);
}

// Ritz vector from the stored Krylov basis: y = sum_k z_k v_k; st->tmp = ||y||.
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_ritz(const val_t<VC>* __restrict__ basis,
                                                 const double* __restrict__ z, int n,
                                                 int64_t dim, val_t<VC>* __restrict__ y,
                                                 LancState* st, RedSlot slot) {
  using V = val_t<VC>;
  double part = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim;
       i += (int64_t)gridDim.x * kBlock) {
    V acc = vzero<V>();
    for (int k = 0; k < n; k++) acc = add(acc, scl(z[k], basis[(int64_t)k * dim + i]));
    y[i] = acc;
    part += redot(acc, acc);
  }
  double tot;
  if (grid_reduce_last(part, slot, &tot) && threadIdx.x == 0) st->tmp = sqrt(tot);
}

// y += z * P (second-pass Ritz accumulation when the basis is not kept)
template <bool VC>
__global__ void __launch_bounds__(kBlock) k_axpy_p(const val_t<VC>* __restrict__ P,
                                                   const double* __restrict__ z, int k,
                                                   int64_t dim, val_t<VC>* __restrict__ y) {
  const double c = z[k];
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim;
       i += (int64_t)gridDim.x * kBlock)
    y[i] = add(y[i], scl(c, P[i]));
}

template <bool VC>
__global__ void __launch_bounds__(kBlock) k_norm(const val_t<VC>* __restrict__ y, int64_t dim,
                                                 LancState* st, RedSlot slot) {
  double part = 0.0;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim;
       i += (int64_t)gridDim.x * kBlock)
    part += redot(y[i], y[i]);
  double tot;
  if (grid_reduce_last(part, slot, &tot) && threadIdx.x == 0) st->tmp = sqrt(tot);
}

template <bool VC>
__global__ void __launch_bounds__(kBlock) k_scale_tmp(val_t<VC>* __restrict__ y, int64_t dim,
                                                      const LancState* st) {
  const double n = st->tmp;
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < dim;
       i += (int64_t)gridDim.x * kBlock) {
    auto v = y[i];
    if constexpr (VC) y[i] = make_double2(v.x / n, v.y / n);
    else y[i] = v / n;
  }
}

}  // namespace edg
