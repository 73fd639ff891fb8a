// ed_lib.hip — the C-ABI of include/ed_gpu.h on top of ed_kernels.hpp.
//
// Sector object = what the reference keeps in module state between
// build_Hv_sector and delete_Hv_sector (ED_HAMILTONIAN_SHARED.f90:32-34,
// ED_VARS_GLOBAL.f90:104-105): the basis H%map, the stored H spH0 (here a
// device SELL-64 matrix) or the matrix-free kernel's tables, plus the
// device-resident Lanczos workspace.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <functional>
#include <mutex>
#include <thread>
#include <string>
#include <map>
#include <vector>

#include "ed_kernels.hpp"
#include "ed_persist.hpp"
#include "ed_trlan.hpp"
#include "ed_trlbatch.hpp"
#include "ed_trlmulti.hpp"
#include "ed_fused.hpp"
#include "ed_split.hpp"
#include "ed_tables.hpp"
#include "ed_host.hpp"

using namespace edg;

// ------------------------------------------------------------------ errors
// (fail / HIPCK / CK in ed_host.hpp; the message slot is this TU's)
std::string& ed_err_slot() {
  static thread_local std::string e;
  return e;
}

static constexpr int kMaxGrid = 65536;
// columns of the thick-restart coefficient buffers (ncv + probe columns)
static constexpr int kTrlanMaxCols = 64;  // one thread per row up to 16.7 M rows
static inline int grid_for(int64_t nthreads) {
  int64_t b = (nthreads + kBlock - 1) / kBlock;
  return (int)std::max<int64_t>(1, std::min<int64_t>(b, kMaxGrid));
}
// one-off grid reductions (in-kernel ticket): few enough blocks that the
// ticket word does not serialise (grid-strided kernels)
static inline int grid_once(int64_t nthreads) { return std::min(grid_for(nthreads), 512); }
// Blocks of `fn` the whole chip holds at once (occupancy x CUs, a multiple of
// the 8 XCDs): the grid of a grid-strided kernel whose blocks have equal
// work, so that no block waits for a second round (a 2,048-block grid at 5
// resident blocks per CU runs 1,280 + 768).
static int resident_grid(const void* fn, int block, size_t lds = 0) {
  static std::mutex mu;
  static std::map<std::pair<const void*, size_t>, int> cache;
  std::lock_guard<std::mutex> lk(mu);
  auto it = cache.find({fn, lds});
  if (it != cache.end()) return it->second;
  int per = 0, dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, fn, block, lds) != hipSuccess)
    return 1024;
  const int g = std::max(8, (std::max(per, 1) * ncu) & ~7);
  cache[{fn, lds}] = g;
  return g;
}

// -------------------------------------------------------------- sector obj
struct KronHost {
  int64_t dimup = 0, dimdw = 0;
  int degup = 0, degdw = 0, nimp = 0;
  bool diag_real = true;  // spin-factor diagonals have no imaginary part
  int32_t *upc = nullptr, *dwc = nullptr;
  void *upv = nullptr, *dwv = nullptr, *aup = nullptr, *adw = nullptr;
  double* uimp = nullptr;
  uint8_t *impu = nullptr, *impd = nullptr;
  // two-pass form (k_kron_up + k_kron_dw): up-hop words {col:16 | value index:8}
  bool two = false;
  int cpt = 0, degU = 0, degD = 0;  // template values: columns per thread, slot bounds
  uint32_t *upw = nullptr, *dwo = nullptr;
  uint8_t* dwi = nullptr;
  void *updict = nullptr, *dwdict = nullptr;
  int nupdict = 0, ndwdict = 0;
};

struct LancWS {
  int vc = -1;
  int cap = 0;                  // alpha/beta capacity
  void *R = nullptr, *P = nullptr, *W = nullptr, *Y = nullptr;
  LancState* st = nullptr;
  double* partials = nullptr;   // [kMaxGrid]
  unsigned int* counter = nullptr;
  double *alpha = nullptr, *beta = nullptr, *z = nullptr;  // one block: alpha | beta | z, cap+2 each
  double* h_ab = nullptr;       // pinned host staging for alpha | beta (2*(cap+2))
  hipEvent_t ev[2] = {nullptr, nullptr};  // lanc_run timing
  void* basis = nullptr;
  int basis_cols = 0;
};

struct ed_sector {
  int device = 0;
  std::mutex build_mu;  // lazy table builds (ensure_direct)
  hipStream_t stream = nullptr;  // private stream for synchronous entry points
  bool own_stream = true;        // false: the caller's stream (ed_sector_create's argument)
  EdModel Mh;
  EdModel* Md = nullptr;
  SectorTables T;
  int flags = 0;
  int opts = 0;        // ED_OPT_* kernel alternatives (ed_sector_set_options)
  bool hc = true;      // complex H values
  int64_t dim = 0, nslice = 0;
  // rows of the operator held here: [row0, row0+nrows) of the sector (the
  // reference's MPI row split, ED_HAMILTONIAN.f90:55-62); whole sector: 0, dim
  int64_t row0 = 0, nrows = 0;
  int32_t* d_off = nullptr;
  uint32_t* d_rank = nullptr;
  uint32_t* d_map = nullptr;
  // stored (SELL-64)
  void* d_diag = nullptr;
  int64_t* d_sptr = nullptr;
  int32_t* d_cols = nullptr;
  void* d_vals = nullptr;
  uint16_t* d_cnt = nullptr;
  int64_t nnz = 0, padded = 0;
  // packed stored H (real values, <= 256 distinct): {col:24 | index:8} words
  uint32_t* d_words = nullptr;
  void* d_pdict = nullptr;   // real(8) or complex(8) values (hc)
  int npdict = 0;
  // two-segment stored H (ed_split.hpp): A words (diagonal + in-block
  // elements, row order), B slices (cross-block elements: U list + L words)
  bool split = false;
  int64_t* d_sptrA = nullptr;
  uint32_t* d_wordsA = nullptr;
  int64_t paddedA = 0;
  int wA_max = 0, wA_min = 0;  // widest / narrowest A slice (k_spmv_sa chunk choice)
  int64_t split_meta = 0, split_listR = 0;  // (ed_sector_info.split_bytes)
  int split_uch = 8;        // U batch of k_spmv_sb (7 or 8)
  SplitSlice* d_bsl = nullptr;
  int nbsl = 0;
  // k_spmv_sb work lists (half-chunk-major), each cut into 8 per-XCD ranges:
  // real vectors: items of two 64-row halves of pair slices + the generic
  // slices; complex vectors: every half
  int2* d_itR = nullptr;
  int* d_glist = nullptr;
  int* d_xoff = nullptr;    // [27]: items R | generic | items C ranges
  int2* d_ul = nullptr;
  uint32_t* d_lw = nullptr;
  int64_t nul = 0, nlw = 0, nfar = 0, nfar_u = 0;  // U entries, L words, cross-block elements (all / in U)
  // fused one-pass re-laid stored H (ed_fused.hpp): 64-row units of one idw
  // block with A words (in-block), U list (unit-uniform cross-block), L words
  bool fused = false;
  FuUnit* d_fu = nullptr;
  int64_t nfu = 0;
  uint32_t* d_fa = nullptr;
  int2* d_ful = nullptr;
  uint32_t* d_flw = nullptr;
  int64_t fu_na = 0, fu_nu = 0, fu_nl = 0, fu_far = 0, fu_far_u = 0;  // A words, U entries, L words, cross (all / U)
  int fu_wa_max = 0, fu_wa_min = 0, fu_uch = kFuUChunk;
  // matrix-free, generic (k_direct): chunk list, per-block op lists, 16-bit tables
  DirChunk* d_dchunk = nullptr;   // 64-row chunks (real vectors)
  int ndchunk = 0;
  DirChunk* d_dchunk2 = nullptr;  // 128-row chunks (complex vectors, two rows per lane)
  int ndchunk2 = 0;
  DirGroup* d_dops = nullptr;
  uint16_t *d_rank16 = nullptr, *d_pat16 = nullptr;
  void* d_ddiag = nullptr;   // gen_diag of the sector object's rows (k_gen_diag)
  bool dir_patlds = false;
  int dir_lds = 0, dir_grid = 0;
  // matrix-free, Kronecker form
  bool kron = false;
  KronHost K;
  // host-pointer H·v staging
  void *d_x = nullptr, *d_y = nullptr;
  LancWS ws;
  int64_t bytes = 0;
  std::vector<void*> allocs;
  // persistent one-workgroup Lanczos (small sectors)
  double pthresh = 0.0;     // breakdown threshold of the current persistent run
  // register-resident stored matrix for the persistent kernel (MODE 2)
  int preg_E = 0;           // 0 not built, -1 ineligible, else ELL row width W
  int preg_rpt = 0;         // rows per thread (template value)
  int kreg_W = 0, kreg_rpt = 0;  // MODE 3 (Kronecker words in registers)
  uint32_t* d_pk = nullptr;
  void* d_dict = nullptr;
  int ndict = 0;
  // Kronecker register layout for the persistent kernel (MODE 4)
  int pkr_state = 0;        // 0 not tried, -1 ineligible, 1 tables ready
  int pkr_src = -1;         // path the tables came from (0 stored SELL, 2 hop tables)
  int pkr_E = 0, pkr_rpt = 0, pkr_du = 0, pkr_dd = 0, pkr_degu = 0, pkr_degd = 0;
  const int32_t *d_kupc = nullptr, *d_kdwc = nullptr;
  const double *d_kupv = nullptr, *d_kdwv = nullptr, *d_kdiag = nullptr;
  // graph cache for Lanczos iterations
  hipGraphExec_t gexec = nullptr;
  int g_path = -2, g_vc = -1, g_chunk = 0;
  bool g_basis = false;
};

// All device memory and copies of a sector are ordered on its private stream
// (stream-ordered allocator, async copies + a stream sync): no call here
// synchronises the device or the null stream, so sectors can be built,
// solved (graph capture included) and freed from several host threads at
// once (farm workers).
static int dcopy(const ed_sector* s, void* dst, const void* src, size_t n, hipMemcpyKind k) {
  HIPCK(hipMemcpyAsync(dst, src, n, k, s->stream));
  HIPCK(hipStreamSynchronize(s->stream));
  return ED_OK;
}
static int dalloc(ed_sector* s, void** p, size_t n) {
  if (n == 0) n = 16;
  hipError_t e = hipMallocAsync(p, n, s->stream);
  if (e != hipSuccess) {
    *p = nullptr;
    return fail(e == hipErrorOutOfMemory ? ED_ERR_OOM : ED_ERR_HIP,
                std::string("hipMalloc(") + std::to_string(n) + ") -> " + hipGetErrorString(e));
  }
  s->allocs.push_back(*p);
  s->bytes += (int64_t)n;
  return ED_OK;
}
static void dfree(ed_sector* s, void** p, size_t n) {
  if (!*p) return;
  auto it = std::find(s->allocs.begin(), s->allocs.end(), *p);
  if (it != s->allocs.end()) s->allocs.erase(it);
  (void)hipFreeAsync(*p, s->stream);
  s->bytes -= (int64_t)n;
  *p = nullptr;
}
template <class T>
static int dalloc_t(ed_sector* s, T** p, size_t count) {
  return dalloc(s, (void**)p, count * sizeof(T));
}
template <class T>
static int upload(ed_sector* s, T** p, const std::vector<T>& h) {
  CK(dalloc_t(s, p, h.size()));
  return dcopy(s, *p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice);
}

// Pinned host staging (Lanczos alpha|beta copies) from a process-wide pool
// that only grows: hipHostFree / hipHostMalloc synchronise the device, which
// would stall every other worker thread's stream (and break their graph
// captures) each time a sector is closed or resized.
static std::mutex g_pin_mu;
static std::multimap<size_t, void*> g_pin_free;  // free blocks by size
static std::map<void*, size_t> g_pin_size;       // every block ever allocated
static void* pinned_get(size_t n) {
  {
    std::lock_guard<std::mutex> lk(g_pin_mu);
    auto it = g_pin_free.lower_bound(n);
    if (it != g_pin_free.end()) {
      void* p = it->second;
      g_pin_free.erase(it);
      return p;
    }
  }
  n = std::max<size_t>(n, 4096);
  void* p = nullptr;
  if (hipHostMalloc(&p, n, hipHostMallocDefault) != hipSuccess) return nullptr;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pin_size[p] = n;
  return p;
}
static void pinned_put(void* p) {
  if (!p) return;
  std::lock_guard<std::mutex> lk(g_pin_mu);
  g_pin_free.emplace(g_pin_size[p], p);
}

static void sector_free(ed_sector* s) {
  if (!s) return;
  (void)hipSetDevice(s->device);
  if (s->gexec) (void)hipGraphExecDestroy(s->gexec);
  for (hipEvent_t& e : s->ws.ev)
    if (e) (void)hipEventDestroy(e);
  if (s->stream) {
    for (void* p : s->allocs) (void)hipFreeAsync(p, s->stream);
    (void)hipStreamSynchronize(s->stream);
    if (s->own_stream) (void)hipStreamDestroy(s->stream);
  }
  pinned_put(s->ws.h_ab);  // after the stream sync above: no copy into it is in flight
  delete s;
}

// ---------------------------------------------------------- stored build
// Dictionary of the distinct off-diagonal values (device hash of bit
// patterns); when there are at most 256, pack every SELL slot into one word.
static int build_pack(ed_sector* s) {
  const int64_t slots = s->padded;
  if (slots == 0) return ED_OK;
  const bool hc = s->hc;
  const int hw = hc ? 2 : 1;
  unsigned long long* table;
  unsigned int* ovf;
  uint8_t* tidx;
  double2* reps = nullptr;
  HIPCK(hipMallocAsync((void**)&table, kDictTable * 8, s->stream));
  HIPCK(hipMallocAsync((void**)&ovf, 4, s->stream));
  HIPCK(hipMallocAsync((void**)&tidx, kDictTable, s->stream));
  if (hc) HIPCK(hipMallocAsync((void**)&reps, kDictTable * 16, s->stream));
  auto cleanup = [&]() {
    (void)hipFreeAsync(table, s->stream);
    (void)hipFreeAsync(ovf, s->stream);
    (void)hipFreeAsync(tidx, s->stream);
    if (reps) (void)hipFreeAsync(reps, s->stream);
  };
  HIPCK(hipMemsetAsync(table, 0xFF, kDictTable * 8, s->stream));
  HIPCK(hipMemsetAsync(ovf, 0, 4, s->stream));
  if (hc)
    hipLaunchKernelGGL(k_dict_insert_c, dim3(grid_for(slots)), dim3(kBlock), 0, s->stream,
                       (const double2*)s->d_vals, slots, table, reps, ovf);
  else
    hipLaunchKernelGGL(k_dict_insert, dim3(grid_for(slots)), dim3(kBlock), 0, s->stream,
                       (const double*)s->d_vals, slots, table, ovf);
  HIPCK(hipGetLastError());
  std::vector<unsigned long long> ht(kDictTable);
  std::vector<double> hr(hc ? 2 * kDictTable : 0);
  unsigned int hov = 0;
  HIPCK(hipMemcpyAsync(ht.data(), table, kDictTable * 8, hipMemcpyDeviceToHost, s->stream));
  if (hc) HIPCK(hipMemcpyAsync(hr.data(), reps, kDictTable * 16, hipMemcpyDeviceToHost, s->stream));
  HIPCK(hipMemcpyAsync(&hov, ovf, 4, hipMemcpyDeviceToHost, s->stream));
  HIPCK(hipStreamSynchronize(s->stream));
  std::vector<uint8_t> ti(kDictTable, 0);
  std::vector<double> dict;
  for (int h = 0; h < kDictTable && !hov; h++) {
    if (ht[h] == kDictEmpty) continue;
    if (dict.size() == (size_t)256 * hw) {
      hov = 1;
      break;
    }
    ti[h] = (uint8_t)(dict.size() / hw);
    if (hc) {
      dict.push_back(hr[2 * h]);
      dict.push_back(hr[2 * h + 1]);
    } else {
      double v;
      memcpy(&v, &ht[h], 8);
      dict.push_back(v);
    }
  }
  if (hov) {
    cleanup();
    return ED_OK;  // too many distinct values: the plain SELL path serves
  }
  uint32_t* words = nullptr;
  void* pd = nullptr;
  CK(dalloc(s, &pd, 256 * 8 * hw));
  CK(dalloc(s, (void**)&words, slots * 4));
  HIPCK(hipMemsetAsync(pd, 0, 256 * 8 * hw, s->stream));
  HIPCK(hipMemcpyAsync(pd, dict.data(), dict.size() * 8, hipMemcpyHostToDevice, s->stream));
  HIPCK(hipMemcpyAsync(tidx, ti.data(), kDictTable, hipMemcpyHostToDevice, s->stream));
  if (hc)
    hipLaunchKernelGGL(k_dict_pack_c, dim3(grid_for(slots)), dim3(kBlock), 0, s->stream, s->d_cols,
                       (const double2*)s->d_vals, slots, table, reps, tidx, words, ovf);
  else
    hipLaunchKernelGGL(k_dict_pack, dim3(grid_for(slots)), dim3(kBlock), 0, s->stream, s->d_cols,
                       (const double*)s->d_vals, slots, table, tidx, words);
  HIPCK(hipGetLastError());
  HIPCK(hipMemcpyAsync(&hov, ovf, 4, hipMemcpyDeviceToHost, s->stream));
  HIPCK(hipStreamSynchronize(s->stream));
  cleanup();
  if (hov) {  // a 64-bit key collision between two complex values: keep the plain path
    dfree(s, &pd, 256 * 8 * hw);
    dfree(s, (void**)&words, slots * 4);
    return ED_OK;
  }
  s->d_pdict = pd;
  s->d_words = words;
  s->npdict = (int)(dict.size() / hw);
  return ED_OK;
}

// Row-split sectors (ed_sector_create_rows) hold rows [row0, row0+nrows) of
// H: H·v from a whole-sector vector and the CSR dump only.
static int whole_only(const ed_sector* s) {
  if (s->nrows == s->dim) return ED_OK;
  return fail(ED_ERR_UNSUPPORTED, "row-split sector: only ed_sector_hxv_dev[_path] and ed_sector_dump_csr apply");
}

// Bytes of the stored matrix stream (the NT threshold: beyond ~192 MB it
// cannot stay in the 256 MB MALL next to the vectors).
static int64_t stored_mbytes(const ed_sector* s) {
  const int64_t hv = s->hc ? 16 : 8;
  if (s->d_words) return s->padded * 4 + s->nrows * hv;
  return s->padded * (4 + hv) + s->nrows * hv;
}

// ---------------------------------------------------- two-segment stored H
// (ed_split.hpp).  Built for whole packed sectors whose stored matrix does
// not fit the 256 MB Infinity Cache (the sectors whose one-pass kernel pays
// the down-spin re-gathers from HBM).
static constexpr int64_t kSplitMinBytes = (int64_t)192 << 20;

static int build_split(ed_sector* s) {
  const int64_t dim = s->dim, ns = s->nslice;
  const int hw = s->hc ? 2 : 1;
  const int nsp = s->Mh.ns;
  // the dictionary's zero (padding slots); appended when absent
  std::vector<double> dict(256 * hw);
  CK(dcopy(s, dict.data(), s->d_pdict, dict.size() * 8, hipMemcpyDeviceToHost));
  int z = -1;
  for (int k = 0; k < s->npdict && z < 0; k++) {
    bool zero = true;
    for (int h = 0; h < hw; h++) zero = zero && dict[k * hw + h] == 0.0 && !std::signbit(dict[k * hw + h]);
    if (zero) z = k;
  }
  if (z < 0) {
    if (s->npdict >= 256) return ED_OK;  // no room for a zero: the one-pass kernel serves
    z = s->npdict++;
    HIPCK(hipMemsetAsync((double*)s->d_pdict + (size_t)z * hw, 0, 8 * hw, s->stream));
  }
  const uint32_t zpad = (uint32_t)z << kPackShift;
  // ---- segment A: counts, slice widths, offsets, fill
  uint16_t* na;
  int32_t* width;
  int64_t *bsum, *total;
  int* farmax;
  const int64_t nb = (ns + 1023) / 1024;
  HIPCK(hipMallocAsync((void**)&na, dim * sizeof(uint16_t), s->stream));
  HIPCK(hipMallocAsync((void**)&width, ns * sizeof(int32_t), s->stream));
  HIPCK(hipMallocAsync((void**)&bsum, std::max<int64_t>(nb, 1) * sizeof(int64_t), s->stream));
  HIPCK(hipMallocAsync((void**)&total, sizeof(int64_t), s->stream));
  HIPCK(hipMallocAsync((void**)&farmax, sizeof(int), s->stream));
  auto scratch_free = [&]() {
    (void)hipFreeAsync(na, s->stream);
    (void)hipFreeAsync(width, s->stream);
    (void)hipFreeAsync(bsum, s->stream);
    (void)hipFreeAsync(total, s->stream);
    (void)hipFreeAsync(farmax, s->stream);
  };
  HIPCK(hipMemsetAsync(farmax, 0, sizeof(int), s->stream));
  hipLaunchKernelGGL(k_split_count_a, dim3(grid_for(ns * 64)), dim3(kBlock), 0, s->stream, s->d_sptr, s->d_words,
                     s->d_cnt, s->d_map, nsp, dim, ns, na, width, farmax);
  HIPCK(hipGetLastError());
  int hfar = 0;
  HIPCK(hipMemcpyAsync(&hfar, farmax, sizeof(int), hipMemcpyDeviceToHost, s->stream));
  HIPCK(hipStreamSynchronize(s->stream));
  if (hfar > kSplitFarMax) {
    scratch_free();
    return ED_OK;  // rows with more cross-block elements than the build stages: one-pass
  }
  // cross-block elements = nnz - dim - sum(nA) (the U entries cover nfar_u of them)
  unsigned long long sumA = 0;
  {
    unsigned long long* dn;
    HIPCK(hipMallocAsync((void**)&dn, sizeof(unsigned long long), s->stream));
    HIPCK(hipMemsetAsync(dn, 0, sizeof(unsigned long long), s->stream));
    hipLaunchKernelGGL(k_sum_u16, dim3(grid_once(dim)), dim3(kBlock), 0, s->stream, na, dim, dn);
    HIPCK(hipGetLastError());
    HIPCK(hipMemcpyAsync(&sumA, dn, sizeof(sumA), hipMemcpyDeviceToHost, s->stream));
    HIPCK(hipStreamSynchronize(s->stream));
    (void)hipFreeAsync(dn, s->stream);
  }
  const int64_t nfar = s->nnz - dim - (int64_t)sumA;
  CK(dalloc_t(s, &s->d_sptrA, ns + 1));
  hipLaunchKernelGGL(k_scan_blocks, dim3((unsigned)nb), dim3(1024), 0, s->stream, width, ns, s->d_sptrA, bsum);
  hipLaunchKernelGGL(k_scan_spine, dim3(1), dim3(64), 0, s->stream, bsum, nb, total);
  hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(1024), 0, s->stream, s->d_sptrA, ns, bsum, total);
  HIPCK(hipGetLastError());
  int64_t slotsA = 0;
  HIPCK(hipMemcpyAsync(&slotsA, total, sizeof(int64_t), hipMemcpyDeviceToHost, s->stream));
  HIPCK(hipStreamSynchronize(s->stream));
  s->paddedA = slotsA;
  {
    std::vector<int64_t> hp(ns + 1);
    CK(dcopy(s, hp.data(), s->d_sptrA, (ns + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
    int wm = 0;
    int wn = 1 << 30;
    for (int64_t q = 0; q < ns; q++) {
      wm = std::max(wm, (int)((hp[q + 1] - hp[q]) >> 6));
      wn = std::min(wn, (int)((hp[q + 1] - hp[q]) >> 6));
    }
    s->wA_max = wm;
    s->wA_min = wn;
  }
  CK(dalloc_t(s, &s->d_wordsA, std::max<int64_t>(slotsA, 1)));
  hipLaunchKernelGGL(k_split_fill_a, dim3(grid_for(ns * 64)), dim3(kBlock), 0, s->stream, s->d_sptr, s->d_words,
                     s->d_cnt, s->d_map, nsp, dim, ns, s->d_sptrA, s->d_wordsA, zpad);
  HIPCK(hipGetLastError());
  // ---- segment B: slices of <= 64 rows of one block, chunk-major
  const SectorTables& T = s->T;
  const int64_t nblk = (int64_t)T.blk_off.size() - 1;
  int64_t maxlen = 0;
  for (int64_t b = 0; b < nblk; b++) maxlen = std::max(maxlen, T.blk_off[b + 1] - T.blk_off[b]);
  std::vector<SplitSlice> sl;
  const int64_t R = kSplitRows;
  const int64_t nchunk = (maxlen + R - 1) / R;
  std::vector<int32_t> sid(nchunk * nblk, -1);  // slice of (chunk, block)
  for (int64_t c = 0; c * R < maxlen; c++)
    for (int64_t b = 0; b < nblk; b++) {
      const int64_t len = T.blk_off[b + 1] - T.blk_off[b];
      if (c * R >= len) continue;
      sid[c * nblk + b] = (int32_t)sl.size();
      SplitSlice q{};
      q.row0 = (int32_t)(T.blk_off[b] + c * R);
      q.nfl = (int32_t)std::min<int64_t>(R, len - c * R);
      sl.push_back(q);
    }
  const int64_t nsl = (int64_t)sl.size();
  CK(dalloc_t(s, &s->d_bsl, std::max<int64_t>(nsl, 1)));
  CK(dcopy(s, s->d_bsl, sl.data(), nsl * sizeof(SplitSlice), hipMemcpyHostToDevice));
  const int gb = (int)std::min<int64_t>((nsl + 1) / 2, 65536);
  hipLaunchKernelGGL(k_split_b<false>, dim3(gb), dim3(kSplitBuildBlock), 0, s->stream, s->d_sptr, s->d_words, s->d_cnt,
                     s->d_map, nsp, s->d_bsl, nsl, (int2*)nullptr, (uint32_t*)nullptr, zpad);
  HIPCK(hipGetLastError());
  CK(dcopy(s, sl.data(), s->d_bsl, nsl * sizeof(SplitSlice), hipMemcpyDeviceToHost));
  int64_t uo = 0, lo = 0, nfar_u = 0;
  int numax = 0;
  for (const SplitSlice& q : sl) numax = std::max(numax, q.nu);
  // U batch of segment B: 7 where no slice has more (Nlevels=28 half
  // filling: every row has 7 down-spin hops; a batch of 8 gathers the pad)
  const int uch = numax == 7 ? 7 : kSplitChunk;
  s->split_uch = uch;
  for (SplitSlice& q : sl) {
    nfar_u += (int64_t)q.nu * split_n(q);
    q.nu = (q.nu + uch - 1) / uch * uch;  // padded with {0, zero value}
    q.wl = (q.wl + kSplitLChunk - 1) / kSplitLChunk * kSplitLChunk;
    q.uoff = uo;
    q.loff = lo;
    uo += q.nu;
    lo += kSplitRows * (int64_t)q.wl;
  }
  // Default policy: the two-segment form only where (nearly) every
  // cross-block element is uniform over its slice (normal-mode sectors
  // without Jx/Jp: the down-spin hops).  With per-row L words (spin flips,
  // Jx/Jp) it is slower: N28 with Jx/Jp (95.7 % uniform) 0.308 vs 0.283 ms
  // one-pass, nonSU2 N26 (39 %) 0.493 vs 0.380 (profiles/r5).
  if (!(s->flags & ED_SPLIT_ON) && (double)nfar_u < 0.99 * (double)nfar) {
    scratch_free();
    dfree(s, (void**)&s->d_bsl, nsl * sizeof(SplitSlice));
    dfree(s, (void**)&s->d_wordsA, std::max<int64_t>(slotsA, 1) * sizeof(uint32_t));
    dfree(s, (void**)&s->d_sptrA, (ns + 1) * sizeof(int64_t));
    s->paddedA = 0;
    return ED_OK;
  }
  CK(dcopy(s, s->d_bsl, sl.data(), nsl * sizeof(SplitSlice), hipMemcpyHostToDevice));
  // (+ one chunk: a two-slice batch may read a whole chunk at a slice with no U entries)
  CK(dalloc_t(s, &s->d_ul, uo + kSplitChunk));
  HIPCK(hipMemsetAsync(s->d_ul, 0, (uo + kSplitChunk) * sizeof(int2), s->stream));
  CK(dalloc_t(s, &s->d_lw, std::max<int64_t>(lo, 1)));
  hipLaunchKernelGGL(k_split_b<true>, dim3(gb), dim3(kSplitBuildBlock), 0, s->stream, s->d_sptr, s->d_words, s->d_cnt,
                     s->d_map, nsp, s->d_bsl, nsl, s->d_ul, s->d_lw, zpad);
  HIPCK(hipGetLastError());
  // work lists in half-chunk-major order (k_spmv_sb)
  std::vector<int2> itR;
  std::vector<int> gl;
  int pend = -1;
  for (int64_t c64 = 0; c64 < 2 * nchunk; c64++)
    for (int64_t b = 0; b < nblk; b++) {
      const int32_t id = sid[(c64 / 2) * nblk + b];
      if (id < 0) continue;
      const int h = (int)(c64 & 1);
      const SplitSlice& q = sl[id];
      if (64 * h >= split_n(q)) continue;
      const int e = 2 * id + h;
      if (!(split_flags(q) & kSplitPair)) {
        if (h == 0) gl.push_back(id);
        continue;
      }
      if (pend < 0) {
        pend = e;
      } else if (sl[pend >> 1].nu == q.nu && sl[pend >> 1].wl == q.wl) {
        itR.push_back(make_int2(pend, e));
        pend = -1;
      } else {
        itR.push_back(make_int2(pend, -1));
        pend = e;
      }
    }
  if (pend >= 0) itR.push_back(make_int2(pend, -1));
  // per-XCD ranges: eight equal contiguous parts of each list
  std::vector<int> xo(27);
  for (int x = 0; x <= 8; x++) {
    xo[x] = (int)((int64_t)itR.size() * x / 8);
    xo[9 + x] = (int)((int64_t)gl.size() * x / 8);
  }
  if (itR.empty()) itR.push_back(make_int2(0, -1));
  if (gl.empty()) gl.push_back(0);
  CK(upload(s, &s->d_itR, itR));
  // bytes one launch reads besides the U / L entries: segment A's slice
  // pointers and the work list of the real (or complex) form
  s->split_meta = (ns + 1) * 8;
  s->split_listR = (int64_t)itR.size() * 8 + (int64_t)gl.size() * 4 + nsl * (int64_t)sizeof(SplitSlice);
  CK(upload(s, &s->d_glist, gl));
  CK(upload(s, &s->d_xoff, xo));
  scratch_free();
  s->nbsl = (int)nsl;
  s->nul = uo;
  s->nlw = lo;
  s->nfar_u = nfar_u;
  s->nfar = nfar;
  s->split = true;
  return ED_OK;
}

// ---------------------------------------------- fused one-pass stored H
// (ed_fused.hpp).  Built where the two-segment form is considered (whole
// packed sectors beyond the Infinity Cache) and on request (ED_FUSED_ON).
static int build_fused(ed_sector* s) {
  const int hw = s->hc ? 2 : 1;
  const int nsp = s->Mh.ns;
  // the dictionary's zero (padding slots); appended when absent
  std::vector<double> dict(256 * hw);
  CK(dcopy(s, dict.data(), s->d_pdict, dict.size() * 8, hipMemcpyDeviceToHost));
  int z = -1;
  for (int k = 0; k < s->npdict && z < 0; k++) {
    bool zero = true;
    for (int h = 0; h < hw; h++) zero = zero && dict[k * hw + h] == 0.0 && !std::signbit(dict[k * hw + h]);
    if (zero) z = k;
  }
  if (z < 0) {
    if (s->npdict >= 256) return ED_OK;  // no room for a zero: the one-pass kernel serves
    z = s->npdict++;
    HIPCK(hipMemsetAsync((double*)s->d_pdict + (size_t)z * hw, 0, 8 * hw, s->stream));
  }
  const uint32_t zpad = (uint32_t)z << kPackShift;
  // units: <= 64 consecutive rows of one idw block, row order
  const SectorTables& T = s->T;
  const int64_t nblk = (int64_t)T.blk_off.size() - 1;
  std::vector<FuUnit> un;
  for (int64_t b = 0; b < nblk; b++)
    for (int64_t r = T.blk_off[b]; r < T.blk_off[b + 1]; r += 64) {
      FuUnit u{};
      u.row0 = (int32_t)r;
      u.n = (int32_t)std::min<int64_t>(64, T.blk_off[b + 1] - r);
      un.push_back(u);
    }
  const int64_t nu = (int64_t)un.size();
  if (nu == 0) return ED_OK;
  CK(upload(s, &s->d_fu, un));
  int* farmax;  // [0]: largest cross-block count of a row; [2..3]: cross-block total
  HIPCK(hipMallocAsync((void**)&farmax, 16, s->stream));
  HIPCK(hipMemsetAsync(farmax, 0, 16, s->stream));
  const int gb = (int)std::min<int64_t>((nu + 3) / 4, 65536);
  hipLaunchKernelGGL(k_fu_build<false>, dim3(gb), dim3(kFuBuildBlock), 0, s->stream, s->d_sptr, s->d_words, s->d_cnt,
                     s->d_map, nsp, s->d_fu, nu, (uint32_t*)nullptr, (int2*)nullptr, (uint32_t*)nullptr, zpad, farmax,
                     (unsigned long long*)(farmax + 2));
  HIPCK(hipGetLastError());
  int hfar[4] = {0, 0, 0, 0};
  HIPCK(hipMemcpyAsync(hfar, farmax, 16, hipMemcpyDeviceToHost, s->stream));
  CK(dcopy(s, un.data(), s->d_fu, nu * sizeof(FuUnit), hipMemcpyDeviceToHost));
  (void)hipFreeAsync(farmax, s->stream);
  unsigned long long far_all = 0;
  memcpy(&far_all, hfar + 2, 8);
  if (hfar[0] > kFuFarMax) {  // rows with more cross-block elements than the build stages
    dfree(s, (void**)&s->d_fu, nu * sizeof(FuUnit));
    return ED_OK;
  }
  int numax = 0;
  for (const FuUnit& u : un) numax = std::max(numax, u.nu);
  // U batch: 7 where no unit has more (Nlevels=28 half filling: 7 down hops)
  const int uch = numax == 7 ? 7 : kFuUChunk;
  int64_t ao = 0, uo = 0, lo = 0, far_u = 0;
  int wmax = 0, wmin = 1 << 30;
  for (FuUnit& u : un) {
    far_u += (int64_t)u.nu * u.n;
    wmax = std::max(wmax, u.wa);
    wmin = std::min(wmin, u.wa);
    u.nu = (u.nu + uch - 1) / uch * uch;
    u.wl = (u.wl + kFuLChunk - 1) / kFuLChunk * kFuLChunk;
    u.aoff = ao;
    u.uoff = uo;
    u.loff = lo;
    ao += 64 * (int64_t)u.wa;
    uo += u.nu;
    lo += 64 * (int64_t)u.wl;
  }
  // Default policy: only where (nearly) every cross-block element is
  // unit-uniform.  nonSU2 spin flips stay per-lane L words: N26 (41 % in U)
  // 0.394 vs 0.380 ms one-pass for real vectors, 0.556 vs 0.530 complex H
  // (gpurun_out r6c); N28 with Jx/Jp (95.7 %) gains (0.242 vs 0.275).
  if (!(s->flags & ED_FUSED_ON) && (double)far_u < 0.9 * (double)far_all) {
    dfree(s, (void**)&s->d_fu, nu * sizeof(FuUnit));
    return ED_OK;
  }
  CK(dcopy(s, s->d_fu, un.data(), nu * sizeof(FuUnit), hipMemcpyHostToDevice));
  CK(dalloc_t(s, &s->d_fa, std::max<int64_t>(ao, 1)));
  CK(dalloc_t(s, &s->d_ful, uo + kFuUChunk));
  HIPCK(hipMemsetAsync(s->d_ful, 0, (uo + kFuUChunk) * sizeof(int2), s->stream));
  CK(dalloc_t(s, &s->d_flw, std::max<int64_t>(lo, 1)));
  hipLaunchKernelGGL(k_fu_build<true>, dim3(gb), dim3(kFuBuildBlock), 0, s->stream, s->d_sptr, s->d_words, s->d_cnt,
                     s->d_map, nsp, s->d_fu, nu, s->d_fa, s->d_ful, s->d_flw, zpad, (int*)nullptr,
                     (unsigned long long*)nullptr);
  HIPCK(hipGetLastError());
  HIPCK(hipStreamSynchronize(s->stream));
  s->nfu = nu;
  s->fu_far = (int64_t)far_all;
  s->fu_na = ao;
  s->fu_nu = uo;
  s->fu_nl = lo;
  s->fu_far_u = far_u;
  s->fu_wa_max = wmax;
  s->fu_wa_min = wmin;
  s->fu_uch = uch;
  s->fused = true;
  return ED_OK;
}

static int build_stored(ed_sector* s) {
  const int64_t dim = s->nrows, ns = s->nslice;  // rows held by this sector object
  const uint32_t* map = s->d_map + s->row0;
  uint16_t* cnt;
  int32_t* width;
  int64_t* bsum;
  int64_t* total;
  CK(dalloc_t(s, &cnt, dim));
  s->d_cnt = cnt;
  // width/bsum/total are scratch, freed right after the build
  HIPCK(hipMallocAsync((void**)&width, ns * sizeof(int32_t), s->stream));
  int64_t nb = (ns + 1023) / 1024;
  HIPCK(hipMallocAsync((void**)&bsum, std::max<int64_t>(nb, 1) * sizeof(int64_t), s->stream));
  HIPCK(hipMallocAsync((void**)&total, sizeof(int64_t), s->stream));
  CK(dalloc_t(s, &s->d_sptr, ns + 1));
  hipLaunchKernelGGL(k_count, dim3(grid_for(ns * 64)), dim3(kBlock), 0, s->stream, s->Md, map,
                     dim, ns, cnt, width);
  HIPCK(hipGetLastError());
  hipLaunchKernelGGL(k_scan_blocks, dim3((unsigned)nb), dim3(1024), 0, s->stream, width, ns,
                     s->d_sptr, bsum);
  hipLaunchKernelGGL(k_scan_spine, dim3(1), dim3(64), 0, s->stream, bsum, nb, total);
  hipLaunchKernelGGL(k_scan_add, dim3((unsigned)nb), dim3(1024), 0, s->stream, s->d_sptr, ns,
                     bsum, total);
  HIPCK(hipGetLastError());
  int64_t slots = 0;
  HIPCK(hipMemcpyAsync(&slots, total, sizeof(int64_t), hipMemcpyDeviceToHost, s->stream));
  HIPCK(hipStreamSynchronize(s->stream));
  (void)hipFreeAsync(width, s->stream);
  (void)hipFreeAsync(bsum, s->stream);
  (void)hipFreeAsync(total, s->stream);
  s->padded = slots;
  const size_t hv = s->hc ? 16 : 8;
  CK(dalloc(s, &s->d_diag, dim * hv));
  CK(dalloc_t(s, &s->d_cols, slots));
  CK(dalloc(s, &s->d_vals, slots * hv));
  DevIndex idx{s->d_off, s->d_rank, s->T.ns, s->T.nst - 1};
  if (s->hc)
    hipLaunchKernelGGL(k_fill<true>, dim3(grid_for(dim)), dim3(kBlock), 0, s->stream, s->Md,
                       map, dim, idx, s->d_sptr, (double2*)s->d_diag, s->d_cols,
                       (double2*)s->d_vals);
  else
    hipLaunchKernelGGL(k_fill<false>, dim3(grid_for(dim)), dim3(kBlock), 0, s->stream, s->Md,
                       map, dim, idx, s->d_sptr, (double*)s->d_diag, s->d_cols,
                       (double*)s->d_vals);
  HIPCK(hipGetLastError());
  // nnz = dim (diagonal) + sum(cnt), reduced on the device (no D2H of the counts)
  unsigned long long* dn;
  HIPCK(hipMallocAsync((void**)&dn, sizeof(unsigned long long), s->stream));
  HIPCK(hipMemsetAsync(dn, 0, sizeof(unsigned long long), s->stream));
  hipLaunchKernelGGL(k_sum_u16, dim3(grid_once(dim)), dim3(kBlock), 0, s->stream, cnt, dim, dn);
  HIPCK(hipGetLastError());
  unsigned long long hn = 0;
  HIPCK(hipMemcpyAsync(&hn, dn, sizeof(hn), hipMemcpyDeviceToHost, s->stream));
  HIPCK(hipStreamSynchronize(s->stream));
  (void)hipFreeAsync(dn, s->stream);
  s->nnz = dim + (int64_t)hn;
  if (s->dim <= (int64_t)kPackColMask + 1 && !(s->flags & ED_NO_PACK)) CK(build_pack(s));
  if (s->d_words && !s->hc && s->row0 == 0 && s->nrows == s->dim &&
      (stored_mbytes(s) > kSplitMinBytes || (s->flags & ED_SPLIT_ON)) && !(s->flags & ED_NO_SPLIT))
    CK(build_split(s));
  if (s->d_words && s->row0 == 0 && s->nrows == s->dim &&
      (stored_mbytes(s) > kSplitMinBytes || (s->flags & ED_FUSED_ON)) && !(s->flags & ED_NO_FUSED))
    CK(build_fused(s));
  return ED_OK;
}

// ------------------------------------------------ matrix-free (generic)
// Host side of k_direct: the candidates of gen_row (direct_candidates), the
// op list of every idw block (down-only terms resolved per block into a row
// offset and a signed value, terms that cannot act in the block dropped,
// padded to kDirGroup), the 64-row chunks of the held rows and the 16-bit
// rank / by-class pattern tables.
struct RecAcc {
  std::vector<uint32_t> k;
  std::vector<double> re, im;
  double dr = 0.0, di = 0.0;
  void diag(double r, double i) { dr = r; di = i; }
  void off(uint32_t t, double r, double i) {
    k.push_back(t);
    re.push_back(r);
    im.push_back(i);
  }
};
static bool same_bits(double a, double b) { return memcmp(&a, &b, 8) == 0; }

// The candidates must reproduce gen_row element by element (target, value
// bits, order): checked on sample states of the sector before any launch.
static int direct_candidates_check(const ed_sector* s, const std::vector<DirCand>& cands) {
  const SectorTables& T = s->T;
  const int64_t nb = (int64_t)T.blk_idw.size();
  const int64_t step = std::max<int64_t>(1, s->dim / 4096);
  for (int64_t i = 0; i < s->dim; i += step) {
    const int64_t b = std::upper_bound(T.blk_off.begin(), T.blk_off.begin() + nb + 1, i) - T.blk_off.begin() - 1;
    const uint32_t idw = T.blk_idw[b];
    const uint32_t m = T.by_cls[T.cls_start[T.need_cls[idw]] + (i - T.blk_off[b])] | (idw << T.ns);
    RecAcc ref;
    gen_row(s->Mh, m, ref);
    size_t q = 0;
    for (const DirCand& c : cands) {
      uint32_t k;
      double sg;
      if (!cand_apply(c, m, &k, &sg)) continue;
      const double re = c.re * sg, im = c.im_signed ? c.im * sg : c.im;
      if (q >= ref.k.size() || ref.k[q] != k || !same_bits(ref.re[q], re) || !same_bits(ref.im[q], im))
        return fail(ED_ERR_STATE, "direct candidates differ from gen_row (row " + std::to_string(i) + ")");
      q++;
    }
    if (q != ref.k.size()) return fail(ED_ERR_STATE, "direct candidates miss elements of gen_row");
  }
  return ED_OK;
}

// Merge LANE op b into a (previous op of the same block) when they are the two
// directions of one hop: same two flip bits (up levels), same value and
// target block, conditions equal except on the flip bits where they read
// (1,0) and (0,1), and a Jordan-Wigner parity that agrees once the flip bits'
// part of popc(m & smask) is folded into the constant.
static bool dir_merge(DirOp& a, const DirOp& b, uint32_t nst) {
  if (!(a.kind & kDirLane) || (a.kind & kDirXor) || !(b.kind & kDirLane)) return false;
  const uint32_t fl = a.flip;
  if (fl != b.flip || __builtin_popcount(fl) != 2 || (fl & ~(nst - 1)) != 0) return false;
  if (a.delta != b.delta || !same_bits(a.re, b.re) || !same_bits(a.im, b.im) ||
      (a.kind & kDirImSigned) != (b.kind & kDirImSigned) || a.smask != b.smask)
    return false;
  if (a.req_mask != b.req_mask || (a.req_mask & fl) != fl) return false;
  if ((a.req_mask & ~fl & (nst - 1)) != 0) return false;  // (the kernel's single condition form)
  if ((a.req_val & ~fl) != (b.req_val & ~fl)) return false;
  const uint32_t va = a.req_val & fl, vb = b.req_val & fl;
  if (__builtin_popcount(va) != 1 || (va ^ vb) != fl) return false;
  const int pa = (__builtin_popcount(va & a.smask) + ((a.kind & kDirC0) ? 1 : 0)) & 1;
  const int pb = (__builtin_popcount(vb & b.smask) + ((b.kind & kDirC0) ? 1 : 0)) & 1;
  if (pa != pb) return false;
  a.req_mask &= ~fl;
  a.req_val &= ~fl;
  a.smask &= ~fl;
  a.xm = fl;
  a.kind = (a.kind & ~kDirC0) | (pa ? kDirC0 : 0) | kDirXor;
  return true;
}

// Op q of a block (down pattern idw, first row own0) folded into slot j of
// a kernel group: conditions, flip and string mask restricted to the up
// pattern; the sign part fixed by the block's down bits and the string's
// constant multiplied into the value (a sign flip: the same bits as the
// reference's products by +-1).  Pads become UNI ops of value 0 on the
// row's own entry.
static void dir_fold(const DirOp& o, uint32_t idw, int ns, uint32_t nst, int64_t own0, DirGroup& G, int j) {
  const uint32_t um = nst - 1, mdw = idw << ns;
  G.cmask[j] = G.cval[j] = G.flipu[j] = G.smasku[j] = G.xm[j] = G.xv[j] = 0;
  if (o.kind & kDirPad) {
    G.delta[j] = (int32_t)own0;
    G.re[j] = G.im[j] = 0.0;
    return;
  }
  const bool ims = (o.kind & kDirImSigned) != 0;
  int neg;
  if (o.kind & kDirLane) {
    G.lanes |= 1u << j;
    // one condition form: popc((u ^ cval) & cmask) == xv — the op's bit
    // conditions (xv = 0), or a merged hop pair's "exactly one of the two
    // bits" (xv = 1; dir_merge leaves such an op no other up-bit condition)
    G.xm[j] = o.xm & um;
    if (o.kind & kDirXor) {
      G.cmask[j] = o.xm & um;
      G.cval[j] = 0;
      G.xv[j] = 1;
    } else {
      G.cmask[j] = o.req_mask & um;
      G.cval[j] = o.req_val & um;
      G.xv[j] = 0;
    }
    G.flipu[j] = o.flip & um;
    G.smasku[j] = o.smask & um;
    if (ims) G.imsig |= 1u << j;
    neg = (__builtin_popcount(mdw & o.smask) + ((o.kind & kDirC0) ? 1 : 0)) & 1;
  } else {
    neg = (o.kind & kDirC0) ? 1 : 0;  // the block's whole sign (build_direct)
  }
  G.delta[j] = o.delta;
  G.re[j] = neg ? -o.re : o.re;
  G.im[j] = (neg && ims) ? -o.im : o.im;
}

// The kernel's view of op j of a group (host restatement of dir_group):
// fires?, target row, value.
static bool dir_eval(const DirGroup& G, int j, uint32_t up, const std::vector<uint32_t>& rank, int64_t* tgt,
                     double* re, double* im) {
  if (!((G.lanes >> j) & 1u)) {
    *tgt = G.delta[j] + (int64_t)rank[up];
    *re = G.re[j];
    *im = G.im[j];
    return true;
  }
  const bool f = (uint32_t)__builtin_popcount((up ^ G.cval[j]) & G.cmask[j]) == G.xv[j];
  if (!f) return false;
  const bool neg = (__builtin_popcount(up & G.smasku[j]) & 1) != 0;
  *tgt = G.delta[j] + (int64_t)rank[up ^ G.flipu[j]];
  *re = neg ? -G.re[j] : G.re[j];
  *im = (neg && ((G.imsig >> j) & 1u)) ? -G.im[j] : G.im[j];
  return true;
}

// The final kernel groups against gen_row on sample rows: targets (through
// the sector's index), value bits and order (pads: zero products only).
static int direct_ops_check(const ed_sector* s, const std::vector<DirGroup>& groups, const std::vector<uint8_t>& pad,
                            const std::vector<DirChunk>& chunks) {
  const SectorTables& T = s->T;
  const size_t step = std::max<size_t>(1, chunks.size() / 512);
  for (size_t ci = 0; ci < chunks.size(); ci += step) {
    const DirChunk& ch = chunks[ci];
    for (int l = 0; l < ch.n; l += std::max(1, ch.n / 8)) {
      const int64_t row = ch.row + l;
      const uint32_t up = T.by_cls[ch.pat0 + l];
      const uint32_t m = up | (ch.idw << T.ns);
      RecAcc ref;
      gen_row(s->Mh, m, ref);
      size_t q = 0;
      for (int k = ch.op0; k < ch.op0 + ch.nop; k++) {
        const DirGroup& G = groups[k / kDirGroup];
        const int j = k % kDirGroup;
        int64_t tg;
        double re, im;
        if (!dir_eval(G, j, up, T.rank, &tg, &re, &im)) continue;
        if (pad[k]) {
          if (re != 0.0 || im != 0.0 || tg != row) return fail(ED_ERR_STATE, "direct: pad op is not a zero product");
          continue;
        }
        if (q >= ref.k.size() || table_index(T, ref.k[q]) != tg || !same_bits(ref.re[q], re) ||
            !same_bits(ref.im[q], im))
          return fail(ED_ERR_STATE, "direct op lists differ from gen_row (row " + std::to_string(row) + ")");
        q++;
      }
      if (q != ref.k.size()) return fail(ED_ERR_STATE, "direct op lists miss elements of gen_row");
    }
  }
  return ED_OK;
}

static int build_direct(ed_sector* s) {
  const SectorTables& T = s->T;
  const int ns = T.ns;
  const uint32_t nst = T.nst;
  std::vector<DirCand> cands;
  direct_candidates(s->Mh, cands);
  CK(direct_candidates_check(s, cands));
  std::vector<DirOp> ops;
  std::vector<DirChunk> chunks, chunks2;  // 64- and 128-row chunks
  std::vector<std::pair<uint32_t, int64_t>> opblk;  // per op: (idw, first row) of its block
  const int64_t r0 = s->row0, r1 = s->row0 + s->nrows;
  for (size_t b = 0; b + 1 < T.blk_off.size(); b++) {
    const int64_t lo = std::max<int64_t>(T.blk_off[b], r0), hi = std::min<int64_t>(T.blk_off[b + 1], r1);
    if (lo >= hi) continue;
    const uint32_t idw = T.blk_idw[b];
    const uint32_t mdw = idw << ns;
    const int32_t op0 = (int32_t)ops.size();
    for (const DirCand& c : cands) {
      const uint32_t dmask = ~(nst - 1);  // down levels
      if ((mdw & c.req_mask & dmask) != (c.req_val & dmask)) continue;  // cannot act in this block
      const uint32_t idw2 = idw ^ (c.flip >> ns);
      const int32_t off2 = T.off[idw2];
      const bool uni = ((c.req_mask | c.flip | c.smask) & (nst - 1)) == 0;
      DirOp o{};
      if (uni) {
        // no up bits: always fires in this block, the lane's own rank in the
        // target block, the block's Jordan-Wigner sign in c0
        if (off2 < 0) return fail(ED_ERR_STATE, "direct: a down-level term leaves the sector");
        const int neg = (__builtin_popcount(mdw & c.smask) + c.c0) & 1;
        o.delta = off2;
        o.kind = (neg ? kDirC0 : 0) | (c.im_signed ? kDirImSigned : 0);
        o.re = c.re;
        o.im = c.im;
      } else {
        if (off2 < 0) continue;  // no up pattern can reach an empty block
        o.req_mask = c.req_mask;
        o.req_val = c.req_val;
        o.flip = c.flip;
        o.smask = c.smask;
        o.delta = off2;
        o.kind = kDirLane | (c.c0 ? kDirC0 : 0) | (c.im_signed ? kDirImSigned : 0);
        o.re = c.re;
        o.im = c.im;
      }
      // the two directions of a hop (c+_a c_b then c+_b c_a, adjacent in
      // gen_row order, exclusive conditions): one op firing on "exactly one
      // of the two flip bits set" (halves the per-lane op evaluations)
      if (!uni && (int32_t)ops.size() > op0 && dir_merge(ops.back(), o, nst)) continue;
      ops.push_back(o);
    }
    while ((ops.size() - op0) % kDirGroup) {
      DirOp o{};
      o.req_val = 1;  // (m & 0) != 1: never fires
      o.kind = kDirPad;
      ops.push_back(o);
    }
    const int32_t nop = (int32_t)ops.size() - op0;
    opblk.resize(ops.size(), std::make_pair(idw, T.blk_off[b]));
    const int64_t cls0 = T.cls_start[T.need_cls[idw]];
    for (int rr = 0; rr < 2; rr++)
      for (int64_t r = lo; r < hi; r += 64 << rr) {
        DirChunk ch{};
        ch.row = (int32_t)r;
        ch.idw = idw;
        ch.pat0 = (int32_t)(cls0 + (r - T.blk_off[b]));
        ch.n = (int32_t)std::min<int64_t>(64 << rr, hi - r);
        ch.op0 = op0;
        ch.nop = nop;
        (rr ? chunks2 : chunks).push_back(ch);
      }
  }
  std::vector<DirGroup> groups(std::max<size_t>(ops.size() / kDirGroup, 1));  // (valid pointer)
  std::vector<uint8_t> pad(ops.size(), 0);
  for (size_t q = 0; q < ops.size(); q++) {
    dir_fold(ops[q], opblk[q].first, ns, nst, opblk[q].second, groups[q / kDirGroup], (int)(q % kDirGroup));
    pad[q] = (ops[q].kind & kDirPad) ? 1 : 0;
  }
  CK(direct_ops_check(s, groups, pad, chunks));
  std::vector<uint16_t> rk(std::max<uint32_t>(nst, 8), 0), pt(std::max<uint32_t>(nst, 8), 0);
  for (uint32_t x = 0; x < nst; x++) {
    rk[x] = (uint16_t)T.rank[x];
    pt[x] = (uint16_t)T.by_cls[x];
  }
  s->ndchunk = (int)chunks.size();
  s->ndchunk2 = (int)chunks2.size();
  if (chunks.empty()) chunks.resize(1);
  if (chunks2.empty()) chunks2.resize(1);
  CK(upload(s, &s->d_dchunk, chunks));
  CK(upload(s, &s->d_dchunk2, chunks2));

  CK(upload(s, &s->d_dops, groups));
  CK(upload(s, &s->d_rank16, rk));
  CK(upload(s, &s->d_pat16, pt));
  // the rows' diagonal, once (k_direct reads it instead of running gen_diag)
  CK(dalloc(s, &s->d_ddiag, (size_t)std::max<int64_t>(s->nrows, 1) * (s->hc ? 16 : 8)));
  if (s->nrows > 0) {
    if (s->hc)
      hipLaunchKernelGGL(k_gen_diag<true>, dim3(grid_for(s->nrows)), dim3(kBlock), 0, s->stream, s->Md,
                         s->d_map + s->row0, s->nrows, (double2*)s->d_ddiag);
    else
      hipLaunchKernelGGL(k_gen_diag<false>, dim3(grid_for(s->nrows)), dim3(kBlock), 0, s->stream, s->Md,
                         s->d_map + s->row0, s->nrows, (double*)s->d_ddiag);
    HIPCK(hipGetLastError());
  }
  // both tables in LDS up to Ns = 15 (128 KB); at Ns = 16 the rank table
  // alone (128 KB), the row's own pattern then read from H%map
  s->dir_patlds = 4 * (int64_t)rk.size() <= 128 * 1024;
  s->dir_lds = (int)((s->dir_patlds ? 4 : 2) * rk.size());
  // 16 chunks per workgroup and step; at most 2 workgroups per CU: the
  // fixed grid also sizes the per-block partials of fused epilogues
  const int g = (int)std::min<int64_t>((s->ndchunk + 15) / 16, 512);
  s->dir_grid = g >= 8 ? (g & ~7) : std::max(g, 1);
  return ED_OK;
}

// the k_direct tables on first use of path 1 (build_direct), ordered before
// the caller's stream by a sync of the sector's stream
static int ensure_direct(ed_sector* s, int path, hipStream_t caller = nullptr) {
  if (path != 1 || s->nrows == 0) return ED_OK;
  // one builder per sector (two threads' first path-1 H·v would race on the
  // tables); a stream being graph-captured cannot take the build's syncs
  std::lock_guard<std::mutex> lk(s->build_mu);
  if (s->d_dchunk) return ED_OK;
  if (caller) {
    hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
    if (hipStreamIsCapturing(caller, &cs) == hipSuccess && cs != hipStreamCaptureStatusNone)
      return fail(ED_ERR_STATE, "first generic matrix-free H·v inside a graph capture: run one outside first");
  }
  if (!(s->flags & ED_DIRECT)) return fail(ED_ERR_ARG, "generic matrix-free path needs ED_DIRECT");
  CK(build_direct(s));
  HIPCK(hipStreamSynchronize(s->stream));
  return ED_OK;
}

template <bool HC, bool VC, bool PL, class Epi>
static int launch_direct(ed_sector* s, const void* x, Epi epi, hipStream_t st) {
  using V = val_t<VC>;
  // the gathers address x through a 4 GiB buffer resource with 32-bit byte
  // offsets (ld_rsrc): a longer vector would read zeros past the range
  if ((uint64_t)s->dim * sizeof(V) > kDirMaxVecBytes)
    return fail(ED_ERR_UNSUPPORTED, "k_direct: vector of " + std::to_string(s->dim) +
                                        " elements exceeds the 4 GiB gather range (use the stored or Kronecker path)");
  constexpr int R = VC ? kDirRows : 1;
  auto fn = k_direct<HC, VC, PL, R, Epi>;
  // dynamic LDS beyond 64 KB: allow what the 160 KB leave next to the
  // function's static LDS (the epilogue's reduction slots)
  static std::once_flag attr;
  static hipError_t ae = hipSuccess;
  std::call_once(attr, [&]() {
    hipFuncAttributes fa{};
    ae = hipFuncGetAttributes(&fa, (const void*)fn);
    if (ae == hipSuccess)
      ae = hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize,
                               160 * 1024 - (int)fa.sharedSizeBytes);
  });
  if (ae != hipSuccess) {
    (void)hipGetLastError();  // not sticky for later launches
    return fail(ED_ERR_HIP, std::string("k_direct LDS attribute -> ") + hipGetErrorString(ae));
  }
  hipLaunchKernelGGL(fn, dim3(s->dir_grid), dim3(kDirBlock), s->dir_lds, st, (const val_t<HC>*)s->d_ddiag,
                     R == 1 ? s->d_dchunk : s->d_dchunk2, R == 1 ? s->ndchunk : s->ndchunk2,
                     s->d_dops, s->d_rank16, s->d_pat16, s->d_map, s->T.ns, (const V*)x, s->dim, s->row0, epi);
  return ED_OK;
}

// ---------------------------------------------------- Kronecker (normal)
struct HopAcc {
  std::vector<uint32_t> tgt;
  std::vector<double> re, im;
  void diag(double, double) {}
  void off(uint32_t k, double r, double i) {
    tgt.push_back(k);
    re.push_back(r);
    im.push_back(i);
  }
};

// Separable one-body diagonal of one spin species (Himp diag + Hbath diag).
static void spin_diag(const EdModel& M, int sp, uint32_t x, double* re, double* im) {
  const int ss = sp == 0 ? 0 : M.S;
  double r = 0.0, i = 0.0;
  for (int o = 0; o < M.norb; o++) {
    double n = (double)bit(x, o);
    r = r + M.hloc_re[ss][ss][o][o] * n;
    i = i + M.hloc_im[ss][ss][o][o] * n;
    r = r - M.xmu * n;
  }
  if (M.bath != ED_BATH_REPLICA) {
    for (int o = 0; o < M.ne; o++)
      for (int k = 0; k < M.nbath; k++) r = r + M.e[ss][o][k] * (double)bit(x, M.stride[o][k]);
  } else {
    for (int k = 0; k < M.nbath; k++)
      for (int o = 0; o < M.norb; o++) {
        double n = (double)bit(x, M.stride[o][k]);
        r = r + M.hb_re[ss][ss][o][o][k] * n;
        i = i + M.hb_im[ss][ss][o][o][k] * n;
      }
  }
  *re = r;
  *im = i;
}

// Two-pass Kronecker tables (k_kron_up): the up-hop ELL slots as 32-bit words
// {column:16 | index:8} over a dictionary of the distinct values (bit
// patterns: exact).  Only for large sectors (dim >= 2^19; the small ones run
// in the persistent kernels) whose up rows fit the register and LDS budget.
// crossover with the one-pass k_kron on configs[3] sectors: dim 392,040 0.0108
// vs 0.0111 ms, 627,264 0.0223 vs 0.0155 ms (tools/kron2_threshold.py)
static constexpr int64_t kKron2MinDim = (int64_t)1 << 19;
// Slot bound of a template instantiation (8, 12 or 16 hops per row).
static int kron_slot_bound(int deg) { return deg <= 8 ? 8 : deg <= 12 ? 12 : 16; }

static int build_kron_words(ed_sector* s, int sp, const std::vector<int32_t>& cols,
                            const std::vector<double>& vals, int64_t nr, int deg,
                            const std::vector<uint8_t>& nhop) {
  KronHost& K = s->K;
  if (sp == 0) {
    K.two = false;
    if (s->flags & ED_KRON2_OFF) return ED_OK;
    if (s->dim < kKron2MinDim && !(s->flags & ED_KRON2_ON)) return ED_OK;
    if (nr > 8192 || deg > 16 || s->dim >= ((int64_t)1 << 31)) return ED_OK;  // 32-bit element offsets
    if (K.nimp * K.nimp > kKronUimpMax) return ED_OK;                          // U table in LDS
    int cpt = 1;
    while (cpt * kKronUpBlock < nr) cpt *= 2;
    K.cpt = cpt;
    K.degU = kron_slot_bound(deg);
    // the thread's up-hop words live in VGPRs: cpt x DEG of them (4 x 16 at
    // DimUp > 2048 spilled to scratch: 3x slower pass U)
    if (cpt * K.degU > (K.degU == 8 ? 64 : 48)) return ED_OK;
    K.two = true;
  } else {
    if (!K.two) return ED_OK;
    K.two = false;
    if (nr > 65535 || deg > 16) return ED_OK;
    K.degD = kron_slot_bound(deg);
  }
  const int hw = s->hc ? 2 : 1;
  std::map<std::pair<uint64_t, uint64_t>, uint32_t> idx;
  std::vector<double> dict;
  std::vector<uint32_t> words((size_t)deg * nr);
  for (size_t q = 0; q < words.size(); q++) {
    uint64_t x0 = 0, x1 = 0;
    memcpy(&x0, &vals[hw * q], 8);
    if (hw == 2) memcpy(&x1, &vals[2 * q + 1], 8);
    auto it = idx.find({x0, x1});
    uint32_t id;
    if (it == idx.end()) {
      id = (uint32_t)idx.size();
      if (id >= (uint32_t)kKronDictMax) {  // too many distinct values: one-pass k_kron
        K.two = false;
        return ED_OK;
      }
      idx[{x0, x1}] = id;
      for (int c = 0; c < hw; c++) dict.push_back(vals[hw * q + c]);
    } else {
      id = it->second;
    }
    words[q] = (uint32_t)cols[q] | (id << 16);
  }
  void*& dp = sp == 0 ? K.updict : K.dwdict;
  if (sp == 0) {
    CK(upload(s, &K.upw, words));
  } else {
    // pass D layout: [row][DEG slot] target rows (the kernel scales them by
    // its row length) and value indices
    // Slot 0's word also carries the row's hop count in bits 24..31: the
    // padding slots (own row, zero value) trail the hops, and pass D skips
    // them with a wave-uniform branch (Norb=2 rows hold 0..12 hops in 12 slots)
    std::vector<uint32_t> off((size_t)nr * K.degD, 0u);
    std::vector<uint8_t> ix((size_t)nr * K.degD, 0);
    for (int64_t r = 0; r < nr; r++) {
      for (int k = 0; k < deg; k++) {
        const uint32_t wd = words[(size_t)k * nr + r];
        off[(size_t)r * K.degD + k] = wd & 0xffffu;
        ix[(size_t)r * K.degD + k] = (uint8_t)(wd >> 16);
      }
      off[(size_t)r * K.degD] |= (uint32_t)nhop[r] << 24;
    }
    CK(upload(s, &K.dwo, off));
    CK(upload(s, &K.dwi, ix));
  }
  CK(dalloc(s, &dp, dict.size() * 8));
  CK(dcopy(s, dp, dict.data(), dict.size() * 8, hipMemcpyHostToDevice));
  (sp == 0 ? K.nupdict : K.ndwdict) = (int)(dict.size() / hw);
  K.two = true;
  return ED_OK;
}

static int build_kron(ed_sector* s) {
  const SectorTables& T = s->T;
  const EdModel& M = s->Mh;
  KronHost& K = s->K;
  const int nup = T.q1, ndw = T.q2;
  K.dimup = T.dimup;
  K.dimdw = T.dimdw;
  K.nimp = 1 << M.norb;
  const uint32_t mask = T.nst - 1;
  const uint32_t* ups = &T.by_cls[T.cls_start[nup]];  // normal mode: class = popcount
  const uint32_t* dws = &T.by_cls[T.cls_start[ndw]];
  const size_t hv = s->hc ? 16 : 8;
  for (int sp = 0; sp < 2; sp++) {
    const int64_t nr = sp == 0 ? K.dimup : K.dimdw;
    const uint32_t* st = sp == 0 ? ups : dws;
    std::vector<HopAcc> rows(nr);
    int deg = 0;
    for (int64_t r = 0; r < nr; r++) {
      uint32_t m = sp == 0 ? st[r] : (st[r] << M.ns);
      gen_row(M, m, rows[r]);
      deg = std::max<int>(deg, (int)rows[r].tgt.size());
    }
    std::vector<uint8_t> nhop(nr);
    for (int64_t r = 0; r < nr; r++) nhop[r] = (uint8_t)rows[r].tgt.size();
    std::vector<int32_t> cols((size_t)deg * nr);
    std::vector<double> vals((size_t)deg * nr * (s->hc ? 2 : 1), 0.0);
    for (int64_t r = 0; r < nr; r++)
      for (int k = 0; k < deg; k++) {
        size_t q = (size_t)k * nr + r;
        if (k < (int)rows[r].tgt.size()) {
          uint32_t t = rows[r].tgt[k];
          uint32_t loc = sp == 0 ? t : (t >> M.ns);
          if ((sp == 0 && (t >> M.ns) != 0) || (sp == 1 && (t & mask) != 0))
            return fail(ED_ERR_STATE, "kron: hop mixes spin species");
          cols[q] = (int32_t)T.rank[loc];
          if (s->hc) {
            vals[2 * q] = rows[r].re[k];
            vals[2 * q + 1] = rows[r].im[k];
          } else {
            vals[q] = rows[r].re[k];
          }
        } else {
          cols[q] = (int32_t)r;  // padding: own column, zero value
        }
      }
    std::vector<double> a(nr * (s->hc ? 2 : 1));
    std::vector<uint8_t> imp(nr);
    for (int64_t r = 0; r < nr; r++) {
      double re, im;
      spin_diag(M, sp, st[r], &re, &im);
      if (im != 0.0) K.diag_real = false;
      if (s->hc) {
        a[2 * r] = re;
        a[2 * r + 1] = im;
      } else {
        a[r] = re;
      }
      imp[r] = (uint8_t)(st[r] & (uint32_t)(K.nimp - 1));
    }
    int32_t* dc;
    void *dv, *da;
    uint8_t* di;
    CK(upload(s, &dc, cols));
    CK(dalloc(s, &dv, vals.size() * 8));
    CK(dcopy(s, dv, vals.data(), vals.size() * 8, hipMemcpyHostToDevice));
    CK(dalloc(s, &da, a.size() * 8));
    CK(dcopy(s, da, a.data(), a.size() * 8, hipMemcpyHostToDevice));
    CK(upload(s, &di, imp));
    CK(build_kron_words(s, sp, cols, vals, nr, deg, nhop));
    if (sp == 0) {
      K.degup = deg; K.upc = dc; K.upv = dv; K.aup = da; K.impu = di;
    } else {
      K.degdw = deg; K.dwc = dc; K.dwv = dv; K.adw = da; K.impd = di;
    }
    (void)hv;
  }
  std::vector<double> u((size_t)K.nimp * K.nimp);
  for (int x = 0; x < K.nimp; x++)
    for (int y = 0; y < K.nimp; y++) u[(size_t)x * K.nimp + y] = hint_value(M, (uint32_t)x, (uint32_t)y);
  CK(upload(s, &K.uimp, u));
  return ED_OK;
}

template <bool HC>
static KronArgs<HC> kron_args(const ed_sector* s) {
  using H = val_t<HC>;
  KronArgs<HC> a;
  a.dimup = s->K.dimup; a.dimdw = s->K.dimdw; a.degup = s->K.degup; a.degdw = s->K.degdw;
  a.nimp = s->K.nimp;
  a.upc = s->K.upc; a.upv = (const H*)s->K.upv; a.dwc = s->K.dwc; a.dwv = (const H*)s->K.dwv;
  a.aup = (const H*)s->K.aup; a.adw = (const H*)s->K.adw; a.uimp = s->K.uimp;
  a.impu = s->K.impu; a.impd = s->K.impd;
  return a;
}

// ------------------------------------------------------------ H·v launch
// path: 0 = stored SELL, 1 = direct generic, 2 = direct Kronecker, -1 = default
static int resolve_path(const ed_sector* s, int path) {
  if (path == -1) {
    if (s->flags & ED_STORED) return 0;
    return s->kron ? 2 : 1;
  }
  if (path == 0 && !(s->flags & ED_STORED)) return -1;
  if (path == 2 && !s->kron) return -1;
  if (path < 0 || path > 2) return -1;
  return path;
}

// XCD-aware block order for the stored kernels (each XCD sweeps one row
// range, so its L2 serves the v gathers of neighbouring rows): n28 packed
// 0.240 -> 0.230 ms, c4 0.0193 -> 0.0173 ms.  The grid is then a multiple of
// 8; every per-block reduction over an H·v launch must use hxv_blocks().
// Only the packed kernel on grids of >= 1024 blocks gains (plain SELL n28:
// 0.421 -> 0.443 ms with the remap; small grids lose blocks to the rounding).
static bool xcd_on(const ed_sector* s, int path) {
  return path == 0 && s->d_words && grid_for(s->nslice * 64) >= 1024;
}
// pass D of the two-pass Kronecker H·v: a multiple of 8 blocks (XCD column
// chunks), 8 resident per CU
static constexpr int kKronDwGrid = 2048;
static constexpr int kKronDwGrid2 = 1280;  // two columns per lane
// pass U LDS: dictionary + two sets of `rows` staged rows
static constexpr int kKronUpSets = 2;
static size_t kron_up_lds(bool hc, bool vc, int64_t du, int rows) {
  return kKronDictMax * (hc ? 16 : 8) + kKronUimpMax * 8 + kKronUpSets * rows * (size_t)((du + 1) & ~1) * (vc ? 16 : 8);
}
static int kron_up_rows(bool hc, bool vc, int64_t du) { return kron_up_lds(hc, vc, du, 2) <= 160 * 1024 ? 2 : 1; }
static bool kron2_on(const ed_sector* s, int path, int vc) {
  if (path != 2 || !s->K.two) return false;
  return kron_up_lds(s->hc, vc, s->K.dimup, 1) <= 160 * 1024;
}
// pass D grid: kKronDwGrid blocks (a multiple of 8: XCD column chunks).
// Every per-block reduction of a pass-D epilogue is sized by this (through
// hxv_blocks).
// Complex vectors take half the grid: their column chunk V[:, c0:c0+64] is
// twice the bytes, and fewer chunks in flight keep it in L2 (N28 complex
// pass D: 512 blocks 187-193 us, 1024 160 us, 2048 167 us; real: 109, 81, 80).
// The two-column real form (even DimUp) has twice the chunk bytes too and
// takes 1280 blocks, 5 per CU (N28: 2048 0.111 ms, 1536 0.115, 1280 0.104-
// 0.106, 1024 0.104, 768 0.106-0.107; N28b 0.134 / 0.129 / 0.126-0.131 /
// 0.129-0.130 / 0.135; configs[3] (6,6) 0.0150 / 0.0152 / 0.0152-0.0153 /
// 0.0155 / 0.0161 ms).
static int kron_dw_grid(const ed_sector* s, bool vc) {
  if (vc) return kKronDwGrid / 2;
  // (a launch whose pointers are not 16-byte aligned falls back to the
  // one-column form on this same grid: hxv_blocks() must match the launch)
  return s->K.dimup % 2 == 0 ? kKronDwGrid2 : kKronDwGrid;
}
// the two-segment stored kernels serve path 0 unless ED_OPT_STORED_EXACT
// The fused form serves complex(8) vectors, and real vectors where the
// two-segment form is not built (its y round trip stays in the Infinity Cache
// for real vectors: N28 0.182 ms against 0.186 fused, gpurun_out r6b).
static bool fused_on(const ed_sector* s, int path, int vc) {
  return path == 0 && s->fused && !(s->opts & (ED_OPT_STORED_EXACT | ED_OPT_NO_FUSED)) && (vc || !s->split);
}
static bool split_on(const ed_sector* s, int path, int vc = 0) {
  // (real vectors only: with complex(8) vectors x and y do not fit the
  // Infinity Cache together and the split is slower than one pass, N28 0.359
  // against 0.316 ms)
  return path == 0 && s->split && !vc && !(s->opts & ED_OPT_STORED_EXACT);
}
static int fused_grid(const ed_sector* s, int vc);
static int hxv_blocks(const ed_sector* s, int path, int vc = 0) {
  if (kron2_on(s, path, vc)) return kron_dw_grid(s, vc);
  if (fused_on(s, path, vc)) return fused_grid(s, vc);
  if (split_on(s, path, vc)) return kSplitGrid;
  if (path == 1) return s->dir_grid;
  const int g = grid_for(s->nslice * 64);
  return xcd_on(s, path) ? (g & ~7) : g;
}

template <bool HC, bool VC, int CPT, int DEGU, int RU>
static int launch_kron_up_t(ed_sector* s, const void* x, void* y, hipStream_t st, int64_t w0, int64_t nw) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  KronHost& K = s->K;
  const size_t lds = kron_up_lds(HC, VC, K.dimup, RU);
  auto fn = k_kron_up<HC, VC, CPT, DEGU, RU>;
  static thread_local int attr_set = 0;
  if (!attr_set) {
    HIPCK(hipFuncSetAttribute((const void*)fn, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024));
    attr_set = 1;
  }
  static thread_local int up_grid = 0;  // per instantiation and LDS size (occupancy x CUs)
  static thread_local size_t up_lds = 0;
  if (!up_grid || up_lds != lds) {
    up_lds = lds;
    int per = 0, dev = 0, ncu = 0;
    HIPCK(hipGetDevice(&dev));
    HIPCK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
    HIPCK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, (const void*)fn, kKronUpBlock, lds));
    up_grid = std::max(per, 1) * ncu;
  }
  // down rows [w0, w0+nw) (the whole sector, or a rank's row block: x, y
  // are then that block)
  KronArgs<HC> ka = kron_args<HC>(s);
  ka.adw += w0;
  ka.impd += w0;
  ka.dimdw = nw;
  hipLaunchKernelGGL(fn, dim3((int)std::min<int64_t>(nw, up_grid)), dim3(kKronUpBlock), lds, st, ka, K.upw,
                     (const H*)K.updict, K.nupdict, (const V*)x, (V*)y);
  HIPCK(hipGetLastError());
  return ED_OK;
}

template <bool HC, bool VC, int CPT, int DEGU>
static int launch_kron_up(ed_sector* s, const void* x, void* y, hipStream_t st, int64_t w0, int64_t nw) {
  // two staged rows per step when LDS allows, except at 4 columns x > 8 slots
  // per thread, where the second row's registers spill (n28b pass U: 97 us
  // with 2 rows, 67 us with 1)
  if (!(CPT >= 4 && DEGU > 8) && kron_up_rows(HC, VC, s->K.dimup) == 2)
    return launch_kron_up_t<HC, VC, CPT, DEGU, 2>(s, x, y, st, w0, nw);
  return launch_kron_up_t<HC, VC, CPT, DEGU, 1>(s, x, y, st, w0, nw);
}

// pass U over down rows [w0, w0+nw)
template <bool HC, bool VC>
static int launch_kron_up_any(ed_sector* s, const void* x, void* y, hipStream_t st, int64_t w0, int64_t nw) {
  switch (s->K.cpt * 100 + s->K.degU) {
    case 108: return launch_kron_up<HC, VC, 1, 8>(s, x, y, st, w0, nw);
    case 116: return launch_kron_up<HC, VC, 1, 16>(s, x, y, st, w0, nw);
    case 208: return launch_kron_up<HC, VC, 2, 8>(s, x, y, st, w0, nw);
    case 112: return launch_kron_up<HC, VC, 1, 12>(s, x, y, st, w0, nw);
    case 212: return launch_kron_up<HC, VC, 2, 12>(s, x, y, st, w0, nw);
    case 216: return launch_kron_up<HC, VC, 2, 16>(s, x, y, st, w0, nw);
    case 408: return launch_kron_up<HC, VC, 4, 8>(s, x, y, st, w0, nw);
    case 412: return launch_kron_up<HC, VC, 4, 12>(s, x, y, st, w0, nw);
    case 808: return launch_kron_up<HC, VC, 8, 8>(s, x, y, st, w0, nw);
    default: return fail(ED_ERR_STATE, "kron2: no instantiation for this geometry");
  }
}

// pass D with rows of length ld over columns [0, ncols); ypart may be null
template <bool HC, bool VC, class Epi>
static int launch_kron_dw(ed_sector* s, const void* x, const void* ypart, Epi epi, hipStream_t st, int ld,
                          int ncols) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  KronHost& K = s->K;
  const int grid = kron_dw_grid(s, VC);
  if constexpr (!HC && !VC) {
    // two columns per lane (16-byte gathers) where the rows, the column
    // range, both vectors and (plain store: one 16-byte store per lane) the
    // output are 16-byte aligned
    bool a16 = ((uintptr_t)x % 16) == 0 && ((uintptr_t)ypart % 16) == 0;
    if constexpr (std::is_same_v<Epi, EpiStore<VC>>) a16 = a16 && ((uintptr_t)epi.hv % 16) == 0;
    if (ld % 2 == 0 && ncols % 2 == 0 && a16) {
      if (K.degD == 8)
        hipLaunchKernelGGL((k_kron_dw<HC, VC, 8, Epi, 2>), dim3(grid), dim3(kBlock), 0, st, kron_args<HC>(s),
                           K.dwo, K.dwi, (const H*)K.dwdict, K.ndwdict, (const V*)x, (const V*)ypart, epi, ld,
                           ncols);
      else if (K.degD == 12)
        hipLaunchKernelGGL((k_kron_dw<HC, VC, 12, Epi, 2>), dim3(grid), dim3(kBlock), 0, st, kron_args<HC>(s),
                           K.dwo, K.dwi, (const H*)K.dwdict, K.ndwdict, (const V*)x, (const V*)ypart, epi, ld,
                           ncols);
      else
        hipLaunchKernelGGL((k_kron_dw<HC, VC, 16, Epi, 2>), dim3(grid), dim3(kBlock), 0, st, kron_args<HC>(s),
                           K.dwo, K.dwi, (const H*)K.dwdict, K.ndwdict, (const V*)x, (const V*)ypart, epi, ld,
                           ncols);
      HIPCK(hipGetLastError());
      return ED_OK;
    }
  }
  if (K.degD == 8)
    hipLaunchKernelGGL((k_kron_dw<HC, VC, 8, Epi>), dim3(grid), dim3(kBlock), 0, st, kron_args<HC>(s),
                       K.dwo, K.dwi, (const H*)K.dwdict, K.ndwdict, (const V*)x, (const V*)ypart, epi, ld, ncols);
  else if (K.degD == 12)
    hipLaunchKernelGGL((k_kron_dw<HC, VC, 12, Epi>), dim3(grid), dim3(kBlock), 0, st, kron_args<HC>(s),
                       K.dwo, K.dwi, (const H*)K.dwdict, K.ndwdict, (const V*)x, (const V*)ypart, epi, ld, ncols);
  else
    hipLaunchKernelGGL((k_kron_dw<HC, VC, 16, Epi>), dim3(grid), dim3(kBlock), 0, st, kron_args<HC>(s),
                       K.dwo, K.dwi, (const H*)K.dwdict, K.ndwdict, (const V*)x, (const V*)ypart, epi, ld, ncols);
  HIPCK(hipGetLastError());
  return ED_OK;
}

template <bool HC, bool VC, class Epi>
static int launch_kron2(ed_sector* s, const void* x, Epi epi, hipStream_t st) {
  void* y = (void*)epi.scratch();
  CK((launch_kron_up_any<HC, VC>(s, x, y, st, 0, s->K.dimdw)));
  return launch_kron_dw<HC, VC>(s, x, y, epi, st, (int)s->K.dimup, (int)s->K.dimup);
}

// Two-segment stored H·v (ed_split.hpp): segment A (diagonal + in-block
// elements, k_spmv_pk on the A words) writes y into the epilogue's scratch
// vector, segment B adds the cross-block elements and runs the epilogue.
template <bool HC, bool VC, class Epi>
static int launch_split(ed_sector* s, const void* x, Epi epi, hipStream_t st) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  if constexpr (HC || VC) {
    // (split_on(): real H on real vectors only; the complex forms are not instantiated)
    return fail(ED_ERR_STATE, "two-segment stored H·v serves real H on real vectors");
  } else {
    V* y = (V*)epi.scratch();
    const int64_t dim = s->dim, ns = s->nslice;
    const bool nta = (s->paddedA * 4 + dim * (int64_t)sizeof(H)) > kSplitMinBytes;
    // A: rows of exactly 7 in-block elements (Norb=1, Nbath=13 half filling)
    // take 7-slot chunks, rows of <= 8 chunks of 8 slots (fewer padding
    // gathers than 16); two slices per wave
#define ED_SPA(NTV, CH)                                                                                       \
  hipLaunchKernelGGL((k_spmv_sa<HC, VC, NTV, CH, ED_SA_R>),                                                    \
                     dim3(resident_grid((const void*)k_spmv_sa<HC, VC, NTV, CH, ED_SA_R>, kBlock)), dim3(kBlock), 0, st, \
                     (const H*)s->d_diag, s->d_sptrA, s->d_wordsA, (const H*)s->d_pdict, (const V*)x, y, dim, ns)
    if (s->wA_max == 7 && s->wA_min == 7) {
      if (nta) ED_SPA(1, 7);
      else ED_SPA(0, 7);
    } else if (s->wA_max <= 8) {
      if (nta) ED_SPA(1, 8);
      else ED_SPA(0, 8);
    } else if (s->wA_max <= 12) {  // (Norb=2: up to 12 in-block elements per row)
      if (nta) ED_SPA(1, 12);
      else ED_SPA(0, 12);
    } else {
      if (nta) ED_SPA(1, kChunk);
      else ED_SPA(0, kChunk);
    }
#undef ED_SPA
    HIPCK(hipGetLastError());
#define ED_SPB(NTV, U)                                                                                        \
  hipLaunchKernelGGL((k_spmv_sb<HC, VC, NTV, Epi, U>), dim3(kSplitGrid), dim3(kBlock), 0, st, s->d_bsl, s->d_itR, \
                     s->d_xoff, s->d_glist, s->d_xoff + 9, s->d_ul, s->d_lw, (const H*)s->d_pdict, (const V*)x,   \
                     (const V*)y, epi)
    const bool ntb = s->nlw * 4 > kSplitMinBytes;
    if (s->split_uch == 7) {
      if (ntb) ED_SPB(1, 7);
      else ED_SPB(0, 7);
    } else {
      if (ntb) ED_SPB(1, kSplitChunk);
      else ED_SPB(0, kSplitChunk);
    }
#undef ED_SPB
    HIPCK(hipGetLastError());
    return ED_OK;
  }
}

// Fused one-pass re-laid stored H·v (ed_fused.hpp).  Grid: half the
// resident blocks, a multiple of 8 (one unit range per XCD) — 16 waves per
// CU keep the window of units an XCD works on (and the neighbour V rows its
// cross-block gathers read) smaller than the full resident grid does: N28
// complex H 0.281 -> 0.269 ms, complex vectors on real H 0.275 -> 0.262, N28
// Jx/Jp real 0.239 -> 0.228; a quarter measured slower (gpurun_out r6f)
#ifndef ED_FU_GRID_DIV
#define ED_FU_GRID_DIV 2
#endif
static int fused_grid(const ed_sector* s, int vc) {
  const int g = vc ? resident_grid((const void*)k_spmv_fu<false, true, 1, EpiStore<true>, 8, 8>, kBlock)
                   : resident_grid((const void*)k_spmv_fu<false, false, 1, EpiStore<false>, 8, 8>, kBlock);
  (void)s;
  return std::max(8, (g / ED_FU_GRID_DIV) & ~7);
}

template <bool HC, bool VC, class Epi>
static int launch_fused(ed_sector* s, const void* x, Epi epi, hipStream_t st) {
  using V = val_t<VC>;
  using H = val_t<HC>;
  const int g = fused_grid(s, VC);
  const bool nt = (s->fu_na + s->fu_nl) * 4 + s->dim * (int64_t)sizeof(H) > kSplitMinBytes;
#define ED_FU(NTV, CH, U)                                                                                      \
  hipLaunchKernelGGL((k_spmv_fu<HC, VC, NTV, Epi, CH, U>), dim3(g), dim3(kBlock), 0, st, (const H*)s->d_diag,      \
                     s->d_fu, s->nfu, s->d_fa, s->d_ful, s->d_flw, (const H*)s->d_pdict, (const V*)x, epi)
#define ED_FU_CH(NTV, U)                                                   \
  do {                                                                     \
    if (s->fu_wa_max == 7 && s->fu_wa_min == 7) ED_FU(NTV, 7, U);          \
    else if (s->fu_wa_max <= 8 || kFuChMax <= 8) ED_FU(NTV, 8, U);         \
    else if (s->fu_wa_max <= 12 || kFuChMax <= 12) ED_FU(NTV, 12, U);      \
    else ED_FU(NTV, kChunk, U);                                            \
  } while (0)
  if (s->fu_uch == 7) {
    if (nt) ED_FU_CH(1, 7);
    else ED_FU_CH(0, 7);
  } else {
    if (nt) ED_FU_CH(1, kFuUChunk);
    else ED_FU_CH(0, kFuUChunk);
  }
#undef ED_FU_CH
#undef ED_FU
  HIPCK(hipGetLastError());
  return ED_OK;
}

template <bool HC, bool VC, class Epi>
static int launch_hxv_t(ed_sector* s, int path, const void* x, Epi epi, hipStream_t st) {
  using V = val_t<VC>;
  const int64_t dim = s->nrows, ns = s->nslice;  // rows of this object; x is the whole sector vector
  const int g = grid_for(ns * 64);
  const int gx = hxv_blocks(s, path, VC);
  const int xr = xcd_on(s, path) ? 1 : 0;
  const V* xo = (const V*)x + s->row0;  // the rows' own entries
  // non-temporal matrix loads once the matrix cannot stay in the 256 MB MALL
  const bool nt = stored_mbytes(s) > ((int64_t)192 << 20);
  // (segment B's pair items load x and y and store the plain epilogue's Hv
  // = y 16 bytes at a time: an 8-byte aligned view, e.g. a torch slice at an
  // odd offset, takes the one-pass kernel)
  if (fused_on(s, path, VC)) return launch_fused<HC, VC>(s, x, epi, st);
  if (split_on(s, path, VC) && !(((uintptr_t)x | (uintptr_t)epi.scratch()) & 15))
    return launch_split<HC, VC>(s, x, epi, st);
  if (path == 0 && s->d_words) {
    using H = val_t<HC>;
    if (nt)
      hipLaunchKernelGGL((k_spmv_pk<HC, VC, 1, Epi>), dim3(gx), dim3(kBlock), 0, st, (const H*)s->d_diag,
                         s->d_sptr, s->d_words, (const H*)s->d_pdict, (const V*)x, xo, dim, ns, epi, xr);
    else
      hipLaunchKernelGGL((k_spmv_pk<HC, VC, 0, Epi>), dim3(gx), dim3(kBlock), 0, st, (const H*)s->d_diag,
                         s->d_sptr, s->d_words, (const H*)s->d_pdict, (const V*)x, xo, dim, ns, epi, xr);
  } else if (path == 0) {
    if (nt)
      hipLaunchKernelGGL((k_spmv<HC, VC, 1, Epi>), dim3(gx), dim3(kBlock), 0, st,
                         (const val_t<HC>*)s->d_diag, s->d_sptr, s->d_cols,
                         (const val_t<HC>*)s->d_vals, (const V*)x, xo, dim, ns, epi, xr);
    else
      hipLaunchKernelGGL((k_spmv<HC, VC, 0, Epi>), dim3(gx), dim3(kBlock), 0, st,
                         (const val_t<HC>*)s->d_diag, s->d_sptr, s->d_cols,
                         (const val_t<HC>*)s->d_vals, (const V*)x, xo, dim, ns, epi, xr);
  } else if (path == 1) {
    const int rc = s->dir_patlds ? launch_direct<HC, VC, true>(s, x, epi, st)
                                 : launch_direct<HC, VC, false>(s, x, epi, st);
    if (rc != ED_OK) return rc;
  } else if (kron2_on(s, path, VC)) {
    return launch_kron2<HC, VC>(s, x, epi, st);
  } else {
    hipLaunchKernelGGL((k_kron<HC, VC, Epi>), dim3(g), dim3(kBlock), 0, st, kron_args<HC>(s),
                       (const V*)x, dim, ns, epi);
  }
  HIPCK(hipGetLastError());
  return ED_OK;
}

template <bool VC, class Epi>
static int launch_hxv(ed_sector* s, int path, const void* x, Epi epi, hipStream_t st) {
  if (s->hc) {
    if constexpr (VC) return launch_hxv_t<true, true>(s, path, x, epi, st);
    return fail(ED_ERR_ARG, "complex Hamiltonian needs complex vectors (vtype=1)");
  }
  return launch_hxv_t<false, VC>(s, path, x, epi, st);
}

// ------------------------------------------------------------ Lanczos
static void drop_graph(ed_sector* s) {
  // a captured graph bakes in buffer pointers: any workspace reallocation
  // invalidates it
  if (s->gexec) (void)hipGraphExecDestroy(s->gexec);
  s->gexec = nullptr;
}

// P (= v_{k-1}) is read by every row slot of the register-mode persistent
// kernels, padding rows included (a guarded load per row costs spills): it
// has at least kPRegBlock * 10 rows, the padding kept zero by the kernel.
static size_t p_rows(const ed_sector* s) { return (size_t)std::max<int64_t>(s->dim, (int64_t)kPRegBlock * 10); }

static int lanc_prepare(ed_sector* s, int vc, int cap, bool want_basis, int basis_cols) {
  LancWS& w = s->ws;
  const size_t vs = vc ? 16 : 8;
  if (w.vc != vc) {
    drop_graph(s);
    if (w.vc != -1) {  // switching real <-> complex vectors: re-size the vector buffers
      HIPCK(hipStreamSynchronize(s->stream));
      const size_t ovs = w.vc ? 16 : 8;
      dfree(s, &w.R, s->dim * ovs);
      dfree(s, &w.P, p_rows(s) * ovs);
      dfree(s, &w.W, s->dim * ovs);
      dfree(s, &w.Y, s->dim * ovs);
      dfree(s, &w.basis, (size_t)w.basis_cols * s->dim * ovs);
      w.basis_cols = 0;
      CK(dalloc(s, &w.R, s->dim * vs));
      CK(dalloc(s, &w.P, p_rows(s) * vs));
      CK(dalloc(s, &w.W, s->dim * vs));
      CK(dalloc(s, &w.Y, s->dim * vs));
      w.vc = vc;
      goto sized;
    }
    CK(dalloc(s, &w.R, s->dim * vs));
    CK(dalloc(s, &w.P, p_rows(s) * vs));
    CK(dalloc(s, &w.W, s->dim * vs));
    CK(dalloc(s, &w.Y, s->dim * vs));
    CK(dalloc_t(s, &w.st, 1));
    CK(dalloc_t(s, &w.partials, kMaxGrid));
    CK(dalloc_t(s, &w.counter, 4));
    HIPCK(hipMemsetAsync(w.counter, 0, 4 * sizeof(unsigned int), s->stream));  // stream-ordered: s->stream does not sync with the null stream
    w.vc = vc;
  }
sized:
  if (cap > w.cap) {
    drop_graph(s);
    double* blk = nullptr;
    CK(dalloc_t(s, &blk, 3 * ((size_t)cap + 2)));
    w.alpha = blk;
    w.beta = blk + (cap + 2);
    w.z = blk + 2 * ((size_t)cap + 2);
    if (w.h_ab) {
      HIPCK(hipStreamSynchronize(s->stream));  // no copy into the old staging in flight
      pinned_put(w.h_ab);
      w.h_ab = nullptr;
    }
    w.h_ab = (double*)pinned_get(2 * ((size_t)cap + 2) * sizeof(double));
    if (!w.h_ab) return fail(ED_ERR_OOM, "pinned host staging");
    w.cap = cap;
  }
  if (want_basis && basis_cols > w.basis_cols) {
    drop_graph(s);
    CK(dalloc(s, &w.basis, (size_t)basis_cols * s->dim * vs));
    w.basis_cols = basis_cols;
  }
  return ED_OK;
}

// splitmix64 hash start vector in [-1,1) (documented in DESIGN.md; tests reproduce it)
__global__ void k_default_start(double* v, int64_t n) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * kBlock) {
    uint64_t z = (uint64_t)(i + 1) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    v[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
  }
}

template <bool VC>
static int lanc_start(ed_sector* s, double thresh, hipStream_t st) {
  LancWS& w = s->ws;
  RedSlot slot{w.partials, w.counter};
  HIPCK(hipMemsetAsync(w.alpha, 0, 2 * (w.cap + 2) * sizeof(double), st));  // alpha | beta
  hipLaunchKernelGGL(k_lanc_init<VC>, dim3(grid_once(s->dim)), dim3(kBlock), 0, st,
                     (const val_t<VC>*)w.R, (val_t<VC>*)w.P, s->dim, w.st, thresh, slot);
  HIPCK(hipGetLastError());
  return ED_OK;
}

template <bool VC>
static int lanc_iter(ed_sector* s, int path, bool basis, hipStream_t st) {
  LancWS& w = s->ws;
  const int g1 = hxv_blocks(s, path, VC), g2 = grid_for(s->dim);
  const bool two1 = g1 > kTicketMaxBlocks, two2 = g2 > kTicketMaxBlocks;
  EpiLancA<VC> e;
  e.st = w.st;
  e.P = (val_t<VC>*)w.P;
  e.W = (val_t<VC>*)w.W;
  e.basis = basis ? (val_t<VC>*)w.basis : nullptr;
  e.dim = s->dim;
  e.alpha_out = w.alpha;
  e.slot = RedSlot{w.partials, two1 ? nullptr : w.counter};
  CK(launch_hxv<VC>(s, path, w.R, e, st));
  if (two1) hipLaunchKernelGGL(k_lanc_fin_a, dim3(1), dim3(kBlock), 0, st, w.partials, g1, w.st, w.alpha);
  RedSlot slot2{w.partials, two2 ? nullptr : w.counter + 1};
  hipLaunchKernelGGL(k_lanc_b<VC>, dim3(g2), dim3(kBlock), 0, st, (const val_t<VC>*)w.W,
                     (const val_t<VC>*)w.P, (val_t<VC>*)w.R, s->dim, w.st, w.beta, slot2);
  if (two2) hipLaunchKernelGGL(k_lanc_fin_b, dim3(1), dim3(kBlock), 0, st, w.partials, g2, w.st, w.beta);
  HIPCK(hipGetLastError());
  return ED_OK;
}

// Run n iterations on stream st; graph-captured in chunks when st is the
// sector's private stream (launch-bound small sectors).
template <bool VC>
static int lanc_iters(ed_sector* s, int path, bool basis, int n, hipStream_t st) {
  const int chunk = 32;
  if (st != s->stream || n < chunk) {
    for (int k = 0; k < n; k++) CK((lanc_iter<VC>(s, path, basis, st)));
    return ED_OK;
  }
  if (!s->gexec || s->g_path != path || s->g_vc != (int)VC || s->g_basis != basis ||
      s->g_chunk != chunk) {
    if (s->gexec) {
      (void)hipGraphExecDestroy(s->gexec);
      s->gexec = nullptr;
    }
    hipGraph_t g;
    HIPCK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
    int rc = ED_OK;
    for (int k = 0; k < chunk && rc == ED_OK; k++) rc = lanc_iter<VC>(s, path, basis, st);
    hipError_t e2 = hipStreamEndCapture(st, &g);
    if (rc != ED_OK) return rc;
    HIPCK(e2);
    HIPCK(hipGraphInstantiate(&s->gexec, g, nullptr, nullptr, 0));
    (void)hipGraphDestroy(g);
    s->g_path = path;
    s->g_vc = VC;
    s->g_basis = basis;
    s->g_chunk = chunk;
  }
  int k = 0;
  for (; k + chunk <= n; k += chunk) HIPCK(hipGraphLaunch(s->gexec, st));
  for (; k < n; k++) CK((lanc_iter<VC>(s, path, basis, st)));
  return ED_OK;
}

// ---------------------------------------------- persistent small-sector path
static constexpr int64_t kLdsBudget = 150 * 1024;

// MODE 2 packing (ELL in registers): row i = t + r*kPRegBlock of thread t
// keeps W words {col:17 | dictionary byte offset:14}, W = the smallest of
// 8/12/14/16 >= the longest row, padded with entry (col 0, dict[0] = 0.0).
// The dictionary holds the distinct values by bit pattern: exact.
static int build_preg(ed_sector* s) {
  if (s->preg_E) return s->preg_E;
  s->preg_E = -1;
  const int64_t dim = s->dim, ns = s->nslice, slots = s->padded;
  if (!(s->flags & ED_STORED) || dim > 10 * (int64_t)kPRegBlock) return -1;
  const int hw = s->hc ? 2 : 1;
  std::vector<uint16_t> cnt(dim);
  std::vector<int64_t> sptr(ns + 1);
  std::vector<int32_t> sc(slots);
  std::vector<double> sv(slots * hw);
  HIPCK(hipStreamSynchronize(s->stream));  // SELL arrays come from kernels on s->stream
  CK(dcopy(s, cnt.data(), s->d_cnt, dim * 2, hipMemcpyDeviceToHost));
  CK(dcopy(s, sptr.data(), s->d_sptr, (ns + 1) * 8, hipMemcpyDeviceToHost));
  CK(dcopy(s, sc.data(), s->d_cols, slots * 4, hipMemcpyDeviceToHost));
  CK(dcopy(s, sv.data(), s->d_vals, slots * 8 * hw, hipMemcpyDeviceToHost));
  if (hw == 2) {  // the register modes keep a real diagonal (Hermitian H)
    std::vector<double> dg(dim * 2);
    CK(dcopy(s, dg.data(), s->d_diag, dim * 16, hipMemcpyDeviceToHost));
    for (int64_t i = 0; i < dim; i++)
      if (dg[2 * i + 1] != 0.0) return -1;
  }
  int wmax = 0;
  for (int64_t i = 0; i < dim; i++) wmax = std::max<int>(wmax, cnt[i]);
  int W = 0;
  for (int w : {8, 12, 14, 16})
    if (!W && wmax <= w) W = w;
  if (!W) return -1;
  const int64_t rpt = (dim + kPRegBlock - 1) / kPRegBlock;
  const int RPT = rpt <= 2 ? 2 : rpt <= 4 ? 4 : rpt <= 6 ? 6 : rpt <= 8 ? 8 : 10;
  const uint32_t hs = s->hc ? 16 : 8;
  std::map<std::pair<uint64_t, uint64_t>, uint32_t> idx;
  std::vector<double> dict(hw, 0.0);
  idx[{0, 0}] = 0;
  std::vector<uint32_t> pk((size_t)RPT * W * kPRegBlock, 0u);
  for (int64_t i = 0; i < dim; i++) {
    const int t = (int)(i % kPRegBlock), r = (int)(i / kPRegBlock);
    const int64_t base = sptr[i >> 6] + (i & 63);
    for (int k = 0; k < cnt[i]; k++) {
      const int64_t q = base + 64 * (int64_t)k;
      uint64_t x0 = 0, x1 = 0;
      memcpy(&x0, &sv[hw * q], 8);
      if (hw == 2) memcpy(&x1, &sv[2 * q + 1], 8);
      auto it = idx.find({x0, x1});
      uint32_t id;
      if (it == idx.end()) {
        id = (uint32_t)idx.size();
        if ((id + 1) * hs > kPkOffMask + 1) return -1;
        idx[{x0, x1}] = id;
        for (int c = 0; c < hw; c++) dict.push_back(sv[hw * q + c]);
      } else {
        id = it->second;
      }
      pk[((size_t)r * W + k) * kPRegBlock + t] = (uint32_t)sc[q] | ((id * hs) << kPkColBits);
    }
  }
  CK(dalloc(s, (void**)&s->d_pk, pk.size() * 4));
  CK(dalloc(s, &s->d_dict, dict.size() * 8));
  CK(dcopy(s, s->d_pk, pk.data(), pk.size() * 4, hipMemcpyHostToDevice));
  CK(dcopy(s, s->d_dict, dict.data(), dict.size() * 8, hipMemcpyHostToDevice));
  s->ndict = (int)(dict.size() / hw);
  s->preg_E = W;
  s->preg_rpt = RPT;
  return W;
}

// MODE 4 (Kronecker register layout, ed_persist.hpp): per lane E up-hop
// entries once plus RPT rows x (E down-hop entries, diagonal, r, p, w) must
// stay below the spill-free budget (-Rpass-analysis=kernel-resource-usage:
// E=4/RPT=10 and E=8/RPT=6 compile without scratch).
// complex vectors (1024 threads, <= 128 VGPRs): per row the down-hop byte
// offsets and the complex w and p; the diagonal and the hop values in LDS
// (-Rpass-analysis: E=4 up to 5 rows, E=8 up to 3 rows spill-free)
static int pkr_geom(ed_sector* s, int64_t du, int64_t dd, int degu, int degd) {
  const int deg = std::max(degu, degd);
  const int E = deg <= 4 ? 4 : deg <= 8 ? 8 : 0;
  if (!E || du < 1 || du > kPRegBlock || du * dd != s->dim) return -1;
  const int64_t G = kPRegBlock / du, rpt = (dd + G - 1) / G;
  const int RPT = rpt <= 2 ? 2 : rpt <= 4 ? 4 : rpt <= 6 ? 6 : rpt <= 8 ? 8 : rpt <= 10 ? 10 : 0;
  if (!RPT || !pkr_fits(E, RPT)) return -1;
  s->pkr_E = E;
  s->pkr_rpt = RPT;
  s->pkr_du = (int)du;
  s->pkr_dd = (int)dd;
  s->pkr_degu = degu;
  s->pkr_degd = degd;
  return 1;
}

// MODE 4 up-hop slot order.  Slot e of every lane is gathered by one
// ds_read_b64 per row; its 32-lane halves hit bank pair (g*DimUp + target)
// mod 32 (the iw*DimUp part common to a wave's rows drops out, so one order
// serves every row slot r), and each extra distinct address on a bank pair
// costs one LDS cycle.  The up list of iu is shared by the G lanes (g, iu):
// permute each list (all orders for E=4, pairwise swaps for E=8) to minimise
// the summed conflict cycles over the halves containing one of its lanes.
// Entries stay the same (target, value) pairs, so H is unchanged; only the
// per-row summation order moves.  configs[1]: 1150 -> ~890 LDS cycles/step.
using PkrHop = std::pair<int32_t, uint64_t>;
static void pkr_order_up(std::vector<std::vector<PkrHop>>& ul, int du, int E) {
  const int G = kPRegBlock / du;
  for (auto& l : ul) l.resize(E, PkrHop{0, 0});  // padding: (col 0, 0.0) reads the row base
  auto half_cost = [&](int h, int e) {
    int nb[32] = {0}, cyc = 0;
    int seen[32][32];
    for (int l = 0; l < 32; l++) {
      const int t = 32 * h + l;
      if (t >= G * du) break;
      const int g = t / du, iu = t - g * du;
      const int addr = g * du + ul[iu][e].first, b = addr & 31;
      bool dup = false;
      for (int k = 0; k < nb[b]; k++) dup |= seen[b][k] == addr;
      if (!dup) { seen[b][nb[b]++] = addr; cyc = std::max(cyc, nb[b]); }
    }
    return cyc;
  };
  auto cost_of = [&](int iu) {
    int c = 0;
    for (int g = 0; g < G; g++) {
      const int h = (g * du + iu) / 32;
      for (int e = 0; e < E; e++) c += half_cost(h, e);
    }
    return c;
  };
  for (int sweep = 0; sweep < 3; sweep++) {
    bool moved = false;
    for (int iu = 0; iu < du; iu++) {
      std::vector<PkrHop>& l = ul[iu];
      int best = cost_of(iu);
      if (E <= 4) {
        std::vector<PkrHop> cur = l, keep = l;
        std::sort(cur.begin(), cur.end());
        do {
          l = cur;
          const int c = cost_of(iu);
          if (c < best) { best = c; keep = cur; moved = true; }
        } while (std::next_permutation(cur.begin(), cur.end()));
        l = keep;
      } else {
        for (int a = 0; a < E; a++)
          for (int b = a + 1; b < E; b++) {
            std::swap(l[a], l[b]);
            const int c = cost_of(iu);
            if (c < best) { best = c; moved = true; } else { std::swap(l[a], l[b]); }
          }
      }
    }
    if (!moved) break;
  }
}

static int pkr_upload(ed_sector* s, const std::vector<std::vector<PkrHop>>& L, int deg, int64_t n,
                      const int32_t** dc, const double** dv) {
  std::vector<int32_t> c((size_t)std::max(deg, 1) * n, 0);
  std::vector<double> v((size_t)std::max(deg, 1) * n, 0.0);
  for (int64_t r = 0; r < n; r++)
    for (size_t e = 0; e < L[r].size() && (int)e < deg; e++) {
      c[e * n + r] = L[r][e].first;
      memcpy(&v[e * n + r], &L[r][e].second, 8);
    }
  int32_t* pc;
  void* pv;
  CK(upload(s, &pc, c));
  CK(dalloc(s, &pv, v.size() * 8));
  CK(dcopy(s, pv, v.data(), v.size() * 8, hipMemcpyHostToDevice));
  *dc = pc;
  *dv = (const double*)pv;
  return ED_OK;
}

// MODE 4 tables of a stored sector: read back from the stored SELL matrix
// and accepted only when it has the Kronecker form H = D + Hup(x)1 + 1(x)Hdw
// on the DimDw x DimUp view (row = iw*DimUp + iu): every entry of row
// (iw, iu) keeps iw (up hop) or iu (down hop), the up list of iu is the same
// (targets and value bits, in order) in every iw block and the down list of
// iw the same for every iu.  The registers then hold exactly the stored
// values; only the summation order (diag, up, down) differs from k_spmv.
static int build_pkron_stored(ed_sector* s) {
  if (s->pkr_state && s->pkr_src == 0) return s->pkr_state;
  s->pkr_state = -1;
  s->pkr_src = 0;
  if (s->hc || s->Mh.mode != ED_MODE_NORMAL || !(s->flags & ED_STORED)) return -1;
  const int64_t du = s->T.dimup, dd = s->T.dimdw, dim = s->dim, ns = s->nslice, slots = s->padded;
  if (du < 1 || du > kPRegBlock || du * dd != dim) return -1;
  std::vector<uint16_t> cnt(dim);
  std::vector<int64_t> sptr(ns + 1);
  std::vector<int32_t> sc(slots);
  std::vector<double> sv(slots);
  HIPCK(hipStreamSynchronize(s->stream));
  CK(dcopy(s, cnt.data(), s->d_cnt, dim * 2, hipMemcpyDeviceToHost));
  CK(dcopy(s, sptr.data(), s->d_sptr, (ns + 1) * 8, hipMemcpyDeviceToHost));
  CK(dcopy(s, sc.data(), s->d_cols, slots * 4, hipMemcpyDeviceToHost));
  CK(dcopy(s, sv.data(), s->d_vals, slots * 8, hipMemcpyDeviceToHost));
  using Hop = PkrHop;
  std::vector<std::vector<Hop>> ul(du), dl(dd);
  std::vector<char> useen(du, 0), dseen(dd, 0);
  std::vector<Hop> lu, ld;
  for (int64_t i = 0; i < dim; i++) {
    const int64_t iw = i / du, iu = i - iw * du, base = sptr[i >> 6] + (i & 63);
    lu.clear();
    ld.clear();
    for (int k = 0; k < cnt[i]; k++) {
      const int64_t q = base + 64 * (int64_t)k;
      const int64_t c = sc[q], cw = c / du, cu = c - cw * du;
      uint64_t bits;
      memcpy(&bits, &sv[q], 8);
      if (cw == iw && cu != iu) lu.push_back({(int32_t)cu, bits});
      else if (cu == iu && cw != iw) ld.push_back({(int32_t)cw, bits});
      else return -1;
    }
    if (!useen[iu]) { ul[iu] = lu; useen[iu] = 1; } else if (ul[iu] != lu) return -1;
    if (!dseen[iw]) { dl[iw] = ld; dseen[iw] = 1; } else if (dl[iw] != ld) return -1;
  }
  int degu = 0, degd = 0;
  for (auto& l : ul) degu = std::max<int>(degu, (int)l.size());
  for (auto& l : dl) degd = std::max<int>(degd, (int)l.size());
  if (pkr_geom(s, du, dd, degu, degd) < 0) return -1;
  pkr_order_up(ul, (int)du, s->pkr_E);
  s->pkr_degu = s->pkr_E;
  CK(pkr_upload(s, ul, s->pkr_degu, du, &s->d_kupc, &s->d_kupv));
  CK(pkr_upload(s, dl, degd, dd, &s->d_kdwc, &s->d_kdwv));
  s->d_kdiag = (const double*)s->d_diag;
  s->pkr_state = 1;
  return 1;
}

// MODE 4 tables of a matrix-free sector: the Kronecker hop tables themselves
// (diagonal generated in-kernel from aup + adw + U, as k_kron).
static int build_pkron_direct(ed_sector* s) {
  if (s->pkr_state && s->pkr_src == 2) return s->pkr_state;
  s->pkr_state = -1;
  s->pkr_src = 2;
  if (s->hc || !s->kron || !s->K.diag_real) return -1;
  const KronHost& K = s->K;
  if (pkr_geom(s, K.dimup, K.dimdw, K.degup, K.degdw) < 0) return -1;
  // up lists from the hop tables ([deg][DimUp], padded with (own column, 0)),
  // reordered for the LDS banks like the stored ones
  const int64_t du = K.dimup;
  std::vector<int32_t> uc((size_t)K.degup * du);
  std::vector<double> uv((size_t)K.degup * du);
  if (K.degup) {
    CK(dcopy(s, uc.data(), K.upc, uc.size() * 4, hipMemcpyDeviceToHost));
    CK(dcopy(s, uv.data(), K.upv, uv.size() * 8, hipMemcpyDeviceToHost));
  }
  std::vector<std::vector<PkrHop>> ul(du);
  for (int64_t r = 0; r < du; r++)
    for (int e = 0; e < K.degup; e++) {
      uint64_t bits;
      memcpy(&bits, &uv[(size_t)e * du + r], 8);
      ul[r].push_back({uc[(size_t)e * du + r], bits});
    }
  pkr_order_up(ul, (int)du, s->pkr_E);
  s->pkr_degu = s->pkr_E;
  CK(pkr_upload(s, ul, s->pkr_degu, du, &s->d_kupc, &s->d_kupv));
  s->d_kdwc = K.dwc;
  s->d_kdwv = (const double*)K.dwv;
  s->d_kdiag = nullptr;
  s->pkr_state = 1;
  return 1;
}

// Returns the persistent mode (0 stored, 1 Kronecker, 2 stored in registers)
// or -1 when the sector does not fit one workgroup's LDS / register budget.
static int64_t persist_lds(const ed_sector* s, int vc, int mode);
// LDS vector rows of a persistent launch: NT * RPT (padding rows stay zero)
static int64_t persist_vrows(const ed_sector* s, int mode, int vc = 0) {
  switch (mode) {
    case 2: return (int64_t)kPRegBlock * s->preg_rpt;
    case 3: return (int64_t)kPRegBlock * s->kreg_rpt;
    case 4: return (int64_t)kPRegBlock * s->pkr_rpt;
    default: return (int64_t)kPBlock * persist_rpt01(s->dim);
  }
}
// ELL words per lane that compile without scratch (-Rpass-analysis=kernel-resource-usage)
static int persist_mode(ed_sector* s, int vc, int path) {
  const int o = s->opts;
  if (o & ED_OPT_NO_PERSIST) return -1;
  const int64_t vs = vc ? 16 : 8;
  // rows per thread beyond which the register-resident p/w arrays spill
  // (-Rpass-analysis: 0-8 B/lane scratch up to 8 real / 5 complex rows)
  const int64_t rpt_max = (vc || s->hc) ? 5 : 8;
  if (s->dim > rpt_max * (int64_t)kPBlock) return -1;
  int64_t lds = ((persist_vrows(s, 0) * vs + 15) & ~(int64_t)15);
  // MODE 4 (Kronecker register layout, real H): c2 2.2 us/step (real
  // vectors); complex vectors in their 1024-thread form
  if (!(o & (ED_OPT_NO_PKRON | ED_OPT_NO_PREG)) &&
      ((path == 0 && !(o & ED_OPT_PERSIST_STORED) && build_pkron_stored(s) > 0) ||
       (path == 2 && build_pkron_direct(s) > 0)) &&
      (vc == 0 || pkr_fits_c512(s->pkr_E, s->pkr_rpt)) &&
      persist_lds(s, vc, 4) <= kLdsBudget)
    return 4;
  // stored: MODE 2 (ELL entries in registers; c2 4.6 us/step) by default.
  // MODE 0 streams the matrix from L2 through one CU (~40-50 GB/s) and is
  // slower than the graph-captured multi-kernel recurrence (c2: 9.8 vs 8.9
  // us/step): opt-in only (ED_OPT_PERSIST_STORED), for coverage
  if (path == 0) {
    if (o & ED_OPT_PERSIST_STORED) return lds <= kLdsBudget ? 0 : -1;
    if (o & ED_OPT_NO_PREG) return -1;
    // MODE 2: dictionary + v + diagonal in LDS; RPT x W words + RPT x (p, w)
    // in registers (512-thread blocks: 256 VGPRs per lane)
    if (s->dim > 10 * (int64_t)kPRegBlock) return -1;
    const int W = build_preg(s);
    if (W < 0) return -1;
    if (s->preg_rpt * W > preg_cap(s->hc, vc)) return -1;
    if (persist_lds(s, vc, 2) > kLdsBudget) return -1;
    return 2;
  }
  if (path == 2 && !(o & ED_OPT_NO_PREG) && s->dim <= 10 * (int64_t)kPRegBlock) {
    // MODE 3: ELL words generated in-kernel from the hop tables
    const KronHost& K = s->K;
    const int deg = K.degup + K.degdw;
    int W = 0;
    for (int w : {8, 12, 14, 16})
      if (!W && deg <= w) W = w;
    const int64_t rpt = (s->dim + kPRegBlock - 1) / kPRegBlock;
    const int RPT = rpt <= 2 ? 2 : rpt <= 4 ? 4 : rpt <= 6 ? 6 : rpt <= 8 ? 8 : 10;
    const int64_t hs = s->hc ? 16 : 8;
    const int64_t dict = ((int64_t)(K.degup * K.dimup + K.degdw * K.dimdw) + 1) * hs;
    const int cap = preg_cap(s->hc, vc);
    const int64_t vr = (int64_t)kPRegBlock * RPT;
    const int64_t l3 = ((dict + 15) & ~(int64_t)15) + ((vr * vs + 15) & ~(int64_t)15) + ((vr * 8 + 15) & ~(int64_t)15);
    if (W && RPT * W <= cap && dict <= (int64_t)kPkOffMask + 1 && l3 <= kLdsBudget && K.diag_real) {
      s->kreg_W = W;
      s->kreg_rpt = RPT;
      return 3;
    }
  }
  if (path == 2) {
    const KronHost& K = s->K;
    const int64_t hs = s->hc ? 16 : 8;
    lds += (K.dimup + K.dimdw) * (hs + 1 + 32) + (int64_t)(K.degup * K.dimup + K.degdw * K.dimdw) * (hs + 4) +
           (int64_t)K.nimp * K.nimp * 8 + 256;
    return lds <= kLdsBudget ? 1 : -1;
  }
  return -1;
}

static int64_t persist_lds(const ed_sector* s, int vc, int mode) {
  const int64_t vs = vc ? 16 : 8, vr = persist_vrows(s, mode, vc);
  int64_t lds = ((vr * vs + 15) & ~(int64_t)15);
  if (mode == 4) {
    // real vectors: slot-major, RPT slots of NT + 1 elements (k_lanc_persist
    // VSLOT); complex vectors: natural order + the down-hop value table
    if (!vc) return (((vr + vr / kPRegBlock) * vs + 15) & ~(int64_t)15);
    return lds + (int64_t)s->pkr_E * s->pkr_dd * 8;
  }
  if (mode == 2) {
    const int64_t hs = s->hc ? 16 : 8;
    return lds + ((vr * 8 + 15) & ~(int64_t)15) + (((int64_t)s->ndict * hs + 15) & ~(int64_t)15);
  }
  if (mode == 3) {
    const int64_t hs = s->hc ? 16 : 8;
    const int64_t dict = ((int64_t)(s->K.degup * s->K.dimup + s->K.degdw * s->K.dimdw) + 1) * hs;
    return lds + ((vr * 8 + 15) & ~(int64_t)15) + ((dict + 15) & ~(int64_t)15);
  }
  if (mode == 1) {
    const KronHost& K = s->K;
    const int64_t hs = s->hc ? 16 : 8;
    auto al = [](int64_t b) { return (b + 15) & ~(int64_t)15; };
    lds += al(K.dimup * hs) + al(K.dimdw * hs) + al((int64_t)K.degup * K.dimup * hs) +
           al((int64_t)K.degdw * K.dimdw * hs) + al((int64_t)K.degup * K.dimup * 4) +
           al((int64_t)K.degdw * K.dimdw * 4) + al(K.dimup) + al(K.dimdw) + al((int64_t)K.nimp * K.nimp * 8);
  }
  return lds;
}

static PersistGeom persist_geom(const ed_sector* s) {
  PersistGeom g;
  g.dim = s->dim;
  g.preg_E = s->preg_E;
  g.preg_rpt = s->preg_rpt;
  g.kreg_W = s->kreg_W;
  g.kreg_rpt = s->kreg_rpt;
  g.pkr_E = s->pkr_E;
  g.pkr_rpt = s->pkr_rpt;
  return g;
}

// Workspace of a batched persistent launch: nb runs on the same H, run b at
// R + b*ldr, P + b*ldp, st + b, alpha/beta + b*ldab.
struct PersistBatch {
  int nb;
  void *R, *P;
  LancState* st;
  double *alpha, *beta;
  int64_t ldr, ldp, ldab;
};

// Launch `niter` persistent iterations.  first=1 starts from the vector in R.
template <bool VC>
static int persist_iters(ed_sector* s, int mode, bool basis, int niter, int first, hipStream_t st,
                         const PersistBatch* bt = nullptr) {
  LancWS& w = s->ws;
  const int nb = bt ? bt->nb : 1;
  auto fill = [&](auto& r) {
    using RT = std::remove_reference_t<decltype(r)>;
    using HT = std::remove_const_t<std::remove_pointer_t<decltype(r.diag)>>;
    memset(&r, 0, sizeof(RT));
    r.diag = (const HT*)s->d_diag;
    r.sptr = s->d_sptr;
    r.cols = s->d_cols;
    r.vals = (const HT*)s->d_vals;
    r.dim = s->dim;
    r.R = w.R;
    r.P = w.P;
    r.st = w.st;
    r.alpha = w.alpha;
    r.beta = w.beta;
    r.basis = basis ? w.basis : nullptr;
    r.niter = niter;
    r.first = first;
    r.thresh = s->pthresh;
    r.pk = s->d_pk;
    r.dict = (const HT*)s->d_dict;
    r.ndict = s->ndict;
    r.kupc = s->d_kupc;
    r.kupv = s->d_kupv;
    r.kdwc = s->d_kdwc;
    r.kdwv = s->d_kdwv;
    r.kdiag = s->d_kdiag;
    r.kdu = s->pkr_du;
    r.kdd = s->pkr_dd;
    r.kdegu = s->pkr_degu;
    r.kdegd = s->pkr_degd;
    if (bt) {
      r.R = bt->R;
      r.P = bt->P;
      r.st = bt->st;
      r.alpha = bt->alpha;
      r.beta = bt->beta;
      r.basis = nullptr;
      r.ldr = bt->ldr;
      r.ldp = bt->ldp;
      r.ldab = bt->ldab;
    }
  };
  const int64_t lds = persist_lds(s, VC, mode);
  if (s->hc) {
    if constexpr (!VC) return fail(ED_ERR_ARG, "complex H needs complex vectors");
    else {
      PersistRun<true> r;
      fill(r);
      if (mode == 1 || mode == 3) r.K = kron_args<true>(s);
      if (mode == 4) return fail(ED_ERR_UNSUPPORTED, "MODE 4 needs real H");
      return persist_launch(true, true, mode, persist_geom(s), &r, lds, st, nb);
    }
  }
  PersistRun<false> r;
  fill(r);
  if (mode == 1 || mode == 3 || (mode == 4 && s->kron)) r.K = kron_args<false>(s);
  return persist_launch(false, VC, mode, persist_geom(s), &r, lds, st, nb);
}

static int persist_set_thresh(ed_sector* s, double thresh, hipStream_t st) {
  // stream-ordered, no host sync: the threshold travels in the kernel
  // argument, the kernel initialises the LancState fields on its first launch
  s->pthresh = thresh;
  HIPCK(hipMemsetAsync(s->ws.st, 0, sizeof(LancState), st));
  HIPCK(hipMemsetAsync(s->ws.alpha, 0, 2 * (s->ws.cap + 2) * sizeof(double), st));  // alpha | beta
  return ED_OK;
}

// Host tridiagonal eigen-solver (tql2, EISPACK; the same algorithm the
// reference uses for Ritz values, .repo/PLAIN_LANCZOS.f90:427-565).
static double pythag(double a, double b) {
  double p = std::max(fabs(a), fabs(b));
  if (p != 0.0) {
    double r = std::min(fabs(a), fabs(b)) / p;
    r = r * r;
    for (;;) {
      double t = 4.0 + r;
      if (t == 4.0) break;
      double s = r / t, u = 1.0 + 2.0 * s;
      p = u * p;
      double su = s / u;
      r = (su * su) * r;
    }
  }
  return p;
}
// d[n] diag, e[n] with e[0] ignored (e[i] couples i-1,i); z column-major n x n or null.
// FAST: hypot in place of EISPACK's iterative pythag (the restart
// eigenproblem of the thick-restart solver; Ritz values of the plain
// Lanczos keep the reference's pythag)
template <bool FAST = false>
static int tql2(int n, double* d, double* e, double* z) {
  if (n == 1) return 0;
  for (int i = 1; i < n; i++) e[i - 1] = e[i];
  e[n - 1] = 0.0;
  double f = 0.0, tst1 = 0.0;
  for (int l = 0; l < n; l++) {
    int j = 0;
    tst1 = std::max(tst1, fabs(d[l]) + fabs(e[l]));
    int m = l;
    for (; m < n; m++)
      if (tst1 + fabs(e[m]) == tst1) break;
    if (m != l) {
      for (;;) {
        if (j >= 30) return l + 1;
        j++;
        int l1 = l + 1, l2 = l1 + 1;
        double g = d[l];
        double p = (d[l1] - g) / (2.0 * e[l]);
        double r = FAST ? hypot(p, 1.0) : pythag(p, 1.0);
        double sr = p >= 0.0 ? fabs(r) : -fabs(r);
        d[l] = e[l] / (p + sr);
        d[l1] = e[l] * (p + sr);
        double dl1 = d[l1];
        double h = g - d[l];
        for (int i = l2; i < n; i++) d[i] -= h;
        f += h;
        p = d[m];
        double c = 1.0, c2 = c, c3 = c, el1 = e[l1], s = 0.0, s2 = 0.0;
        for (int i = m - 1; i >= l; i--) {
          c3 = c2;
          c2 = c;
          s2 = s;
          g = c * e[i];
          h = c * p;
          r = FAST ? hypot(p, e[i]) : pythag(p, e[i]);
          e[i + 1] = s * r;
          s = e[i] / r;
          c = p / r;
          p = c * d[i] - s * g;
          d[i + 1] = h + s * (c * g + s * d[i]);
          if (z)
            for (int k = 0; k < n; k++) {
              h = z[k + (size_t)n * (i + 1)];
              z[k + (size_t)n * (i + 1)] = s * z[k + (size_t)n * i] + c * h;
              z[k + (size_t)n * i] = c * z[k + (size_t)n * i] - s * h;
            }
        }
        p = -s * s2 * c3 * el1 * e[l] / dl1;
        e[l] = s * p;
        d[l] = c * p;
        if (!(tst1 + fabs(e[l]) > tst1)) break;
      }
    }
    d[l] += f;
  }
  for (int ii = 1; ii < n; ii++) {
    int i = ii - 1, k = i;
    double p = d[i];
    for (int jj = ii; jj < n; jj++)
      if (d[jj] < p) { k = jj; p = d[jj]; }
    if (k != i) {
      d[k] = d[i];
      d[i] = p;
      if (z)
        for (int jj = 0; jj < n; jj++) std::swap(z[jj + (size_t)n * i], z[jj + (size_t)n * k]);
    }
  }
  return 0;
}

static double lowest_ritz(const std::vector<double>& a, const std::vector<double>& b, int n) {
  std::vector<double> d(a.begin(), a.begin() + n), e(n, 0.0);
  for (int q = 1; q < n; q++) e[q] = b[q];
  tql2(n, d.data(), e.data(), nullptr);
  return d[0];
}

// ------------------------------------------ thick-restart Lanczos (ARPACK)
// Cyclic Jacobi for a small real symmetric matrix (host): A (n x n, column-
// major) -> ascending eigenvalues w, eigenvectors Z (column-major).
static void jacobi_eigh(int n, std::vector<double> A, std::vector<double>& w, std::vector<double>& Z) {
  Z.assign((size_t)n * n, 0.0);
  for (int i = 0; i < n; i++) Z[i + (size_t)n * i] = 1.0;
  auto a = [&](int i, int j) -> double& { return A[i + (size_t)n * j]; };
  for (int sweep = 0; sweep < 100; sweep++) {
    double off = 0.0, tot = 0.0;
    for (int j = 0; j < n; j++)
      for (int i = 0; i < n; i++) {
        tot += a(i, j) * a(i, j);
        if (i != j) off += a(i, j) * a(i, j);
      }
    if (off <= 1e-30 * tot || off == 0.0) break;
    for (int p = 0; p < n - 1; p++)
      for (int q = p + 1; q < n; q++) {
        const double apq = a(p, q);
        if (apq == 0.0) continue;
        const double theta = (a(q, q) - a(p, p)) / (2.0 * apq);
        const double t = (theta >= 0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
        const double c = 1.0 / sqrt(t * t + 1.0), sn = t * c;
        for (int k = 0; k < n; k++) {  // A <- A J
          const double akp = a(k, p), akq = a(k, q);
          a(k, p) = c * akp - sn * akq;
          a(k, q) = sn * akp + c * akq;
        }
        for (int k = 0; k < n; k++) {  // A <- J^T A
          const double apk = a(p, k), aqk = a(q, k);
          a(p, k) = c * apk - sn * aqk;
          a(q, k) = sn * apk + c * aqk;
        }
        for (int k = 0; k < n; k++) {
          const double zkp = Z[k + (size_t)n * p], zkq = Z[k + (size_t)n * q];
          Z[k + (size_t)n * p] = c * zkp - sn * zkq;
          Z[k + (size_t)n * q] = sn * zkp + c * zkq;
        }
      }
  }
  std::vector<int> idx(n);
  for (int i = 0; i < n; i++) idx[i] = i;
  std::sort(idx.begin(), idx.end(), [&](int x, int y) { return a(x, x) < a(y, y); });
  std::vector<double> Zs((size_t)n * n);
  w.assign(n, 0.0);
  for (int k = 0; k < n; k++) {
    w[k] = a(idx[k], idx[k]);
    for (int i = 0; i < n; i++) Zs[i + (size_t)n * k] = Z[i + (size_t)n * idx[k]];
  }
  Z.swap(Zs);
}

// Householder reduction of a real symmetric matrix to tridiagonal form with
// the transformation accumulated (EISPACK tred2 / Numerical Recipes §11.2):
// A (n x n, column-major, A(i,j) = A[i + n*j]) is overwritten by Q with
// Q^T A Q = tridiag(d, e), e[i] coupling i-1 and i (e[0] = 0).  With tql2
// (same z convention) the projected matrix of a restart costs O(n^3) with a
// small constant: the cyclic Jacobi took ~0.5 ms per 23 x 23 restart on the
// host, most of a small sector's solve.
static void tred2(int n, double* A, double* d, double* e) {
#define TA(i, j) A[(i) + (size_t)n * (j)]
  for (int i = n - 1; i > 0; i--) {
    const int l = i - 1;
    double h = 0.0, scale = 0.0;
    if (l > 0) {
      for (int k = 0; k <= l; k++) scale += fabs(TA(i, k));
      if (scale == 0.0) {
        e[i] = TA(i, l);
      } else {
        for (int k = 0; k <= l; k++) {
          TA(i, k) /= scale;
          h += TA(i, k) * TA(i, k);
        }
        double f = TA(i, l);
        double g = f >= 0.0 ? -sqrt(h) : sqrt(h);
        e[i] = scale * g;
        h -= f * g;
        TA(i, l) = f - g;
        f = 0.0;
        for (int j = 0; j <= l; j++) {
          TA(j, i) = TA(i, j) / h;
          g = 0.0;
          for (int k = 0; k <= j; k++) g += TA(j, k) * TA(i, k);
          for (int k = j + 1; k <= l; k++) g += TA(k, j) * TA(i, k);
          e[j] = g / h;
          f += e[j] * TA(i, j);
        }
        const double hh = f / (h + h);
        for (int j = 0; j <= l; j++) {
          f = TA(i, j);
          e[j] = g = e[j] - hh * f;
          for (int k = 0; k <= j; k++) TA(j, k) -= (f * e[k] + g * TA(i, k));
        }
      }
    } else {
      e[i] = TA(i, l);
    }
    d[i] = h;
  }
  d[0] = 0.0;
  e[0] = 0.0;
  for (int i = 0; i < n; i++) {
    const int l = i - 1;
    if (d[i] != 0.0) {
      for (int j = 0; j <= l; j++) {
        double g = 0.0;
        for (int k = 0; k <= l; k++) g += TA(i, k) * TA(k, j);
        for (int k = 0; k <= l; k++) TA(k, j) -= g * TA(k, i);
      }
    }
    d[i] = TA(i, i);
    TA(i, i) = 1.0;
    for (int j = 0; j <= l; j++) TA(j, i) = TA(i, j) = 0.0;
  }
#undef TA
}

// Symmetric eigenproblem of the projected matrix: ascending w, eigenvectors
// as the columns of Z (column-major).  tred2 + tql2; the cyclic Jacobi only if
// the QL iteration does not converge.
static void sym_eigh(int n, const std::vector<double>& A, std::vector<double>& w, std::vector<double>& Z) {
  Z = A;
  w.assign(n, 0.0);
  std::vector<double> e(n, 0.0);
  tred2(n, Z.data(), w.data(), e.data());
  if (tql2<true>(n, w.data(), e.data(), Z.data()) != 0) jacobi_eigh(n, A, w, Z);
}

__global__ void k_hash_vec(double* v, int64_t n, uint64_t seed) {
  for (int64_t i = (int64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (int64_t)gridDim.x * kBlock) {
    uint64_t z = (uint64_t)(i + 1 + seed * 0x632BE59BD9B4E019ull) * 0x9E3779B97F4A7C15ull;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    v[i] = (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
  }
}

// Thick-restart Lanczos state.  All O(dim) work and the CGS2 coefficients
// stay on the device; one expansion sweep (j0 .. m-1) is captured once per
// start column into a hipGraph (j0 = 0 and j0 = nkeep), so a restart cycle is
// one graph launch + one host sync for the m x m projected problem.
template <bool VC>
struct Trlan {
  using V = val_t<VC>;
  ed_sector* s = nullptr;
  int path = 0;
  hipStream_t st = nullptr;
  int64_t dim = 0;
  int G = 1, m = 0, mcap = 0;  // mcap: basis columns allocated
  bool fused = true;  // false (ED_OPT_TRLAN_UNFUSED): the four-sweep CGS2 (A/B)
  V *Vb = nullptr, *Xb = nullptr, *w = nullptr;
  double2 *h = nullptr, *coef = nullptr, *part = nullptr, *part2 = nullptr;
  // grids up to this fold the coefficient reduction into the next CGS pass
  // (every block re-reads G x ncol partials; 0 with ED_OPT_TRLAN_NOFOLD: A/B)
  // (round 6, in the 8-worker farm: folding at 256 or 512 blocks, with the
  // sweep grid at 512 or 256, within noise of 128, gpurun_out r6k; at the
  // closing build 256 with the 256-block grid: see kTrlanGridCap)
  int kFinFoldG = 256;
  bool graphs_on = true;  // false (ED_OPT_NO_GRAPH): sweeps launched directly
  bool solo = true;       // false (ED_OPT_TRLAN_NOSOLO): multi-kernel CGS on small sectors too (A/B)
  bool locupd = true;     // false (ED_OPT_TRLAN_FULLUPD): full CGS update every step (A/B)
  int* lof = nullptr;     // device: the current step's update was local-only
  double *Y = nullptr, *npart = nullptr, *alpha = nullptr, *beta = nullptr;
  double *npA = nullptr, *npB = nullptr;  // |w|^2 partials before / after the first CGS pass (DGKS)
  double* hp = nullptr;          // pinned staging (trlan_pinned)
  std::vector<void*> mine;
  std::vector<std::pair<int, hipGraphExec_t>> graphs;
  int nhv = 0;
  ~Trlan() {
    for (auto& g : graphs) (void)hipGraphExecDestroy(g.second);
    for (void* p : mine) (void)hipFreeAsync(p, st);
  }
  int alloc(void** p, size_t n) {
    HIPCK(hipMallocAsync(p, n, st));
    mine.push_back(*p);
    return ED_OK;
  }
  V* col(V* b, int c) { return b + (int64_t)c * dim; }
  // x -= V[:, :ncol] V[:, :ncol]^H x, twice; coef = summed coefficients;
  // with jn >= 0: alpha[jn], beta[jn] = ||x|| afterwards
  // one fused sweep (k_cgs) with the column group rounded up to 8/16/24/32
  bool cgs(int ncol, const double2* hin, V* x, double2* pt, double* np, const double2* pin = nullptr,
           int add = 0, const double* dgA = nullptr, const double* dgB = nullptr, int* lf = nullptr,
           const double* locA = nullptr) {
    const int nc = (ncol + 7) / 8 * 8;
#define ED_CGS(NCV) \
  hipLaunchKernelGGL((k_cgs<VC, NCV>), dim3(G), dim3(kBlock), 0, st, Vb, ncol, hin, x, dim, pt, np, pin, G, \
                     coef, add, dgA, dgB, lf, locA)
    if (nc <= 8) ED_CGS(8);
    else if (nc <= 16) ED_CGS(16);
    else if (nc <= 24) ED_CGS(24);
    else if (!VC && nc <= 32) ED_CGS(32);
    else return false;
#undef ED_CGS
    return true;
  }
  // jc: the basis column of v_j when it is not column jn (probe_screen's
  // rolling window; alpha/beta slot jn)
  int orth(int ncol, V* x, int jn, V* out = nullptr, int shifted = 0, int jc = -1) {
    // small sectors: the whole CGS2 + alpha/beta + V_{j+1} in one workgroup
    // (complex vectors: up to 16 columns; the 24/32-column forms spill)
    if (fused && solo && ncol > 0 && dim <= kOrthSoloMaxDim && ncol <= (VC ? 16 : 32)) {
      V* const o = (out && jn >= 0) ? out : nullptr;
      const int js = jn >= 0 ? jn : m;  // beta[m]: scratch slot
      const int nc = (ncol + 7) / 8 * 8;
#define ED_OSOLO(NCV)                                                                                          \
  hipLaunchKernelGGL((k_orth_solo<VC, NCV>), dim3(1), dim3(kOrthSoloBlock), 0, st, Vb, ncol, x, dim, coef,     \
                     jn >= 0 ? alpha : nullptr, beta, jn, js, o, shifted, (shifted && locupd) ? 1 : 0, jc)
      if (nc <= 8) ED_OSOLO(8);
      else if (nc <= 16) ED_OSOLO(16);
      else if constexpr (!VC) {
        if (nc <= 24) ED_OSOLO(24);
        else ED_OSOLO(32);
      }
#undef ED_OSOLO
      return ED_OK;
    }
    // fused CGS: dots + |x|^2 | x -= V h1, dots, |x'|^2 | (DGKS: only if
    // |x'| <= 0.717 |x|) x -= V h2, |x''|^2 — V streamed 2x or 3x
    if (fused && ncol > 0 && cgs(ncol, nullptr, x, part, npA)) {
      // shifted steps: the update may be local-only (cgs_loc_only, decided
      // by the first update pass from the dots and recorded in *lof)
      int* const lf = (shifted && locupd) ? lof : nullptr;
      const double* const la = lf ? npA : nullptr;
      if (G <= kFinFoldG) {
        // small grids: each pass forms the previous pass's coefficients from
        // its partials (k_vdot_fin folded in: 5 launches per step, not 7)
        cgs(ncol, nullptr, x, part2, npB, part, 0, nullptr, nullptr, lf, la);
        cgs(ncol, nullptr, x, nullptr, npart, part2, 1, npA, npB, lf);
      } else {
        hipLaunchKernelGGL(k_vdot_fin<VC>, dim3(ncol), dim3(kBlock), 0, st, part, G, h, coef, 0,
                           (const double*)nullptr, (const double*)nullptr);
        cgs(ncol, h, x, part2, npB, nullptr, 0, nullptr, nullptr, lf, la);
        hipLaunchKernelGGL(k_vdot_fin<VC>, dim3(ncol), dim3(kBlock), 0, st, part2, G, h, coef, 1,
                           (const double*)npA, (const double*)npB);
        cgs(ncol, h, x, nullptr, npart, nullptr, 0, npA, npB, lf);
      }
      if (out && jn >= 0)  // + V_{j+1} = x / beta_j in the same launch
        hipLaunchKernelGGL(k_coef_scale<VC>, dim3(G), dim3(kBlock), 0, st, npart, G, coef, jn, alpha, beta,
                           x, out, dim, shifted, jc);
      else
        hipLaunchKernelGGL(k_trl_coef, dim3(1), dim3(kBlock), 0, st, npart, G, coef, jn >= 0 ? jn : m,
                           jn >= 0 ? alpha : nullptr, beta, jn >= 0 ? shifted : 0, jc);
      return ED_OK;
    }
    if (ncol == 0) {
      hipLaunchKernelGGL(k_vaxpy<VC>, dim3(G), dim3(kBlock), 0, st, Vb, 0, h, x, dim, npart);
    }
    const dim3 gp(G, (ncol + kVCols - 1) / kVCols);
    for (int pass = 0; pass < 2 && ncol > 0; pass++) {
      hipLaunchKernelGGL(k_vdot_part<VC>, gp, dim3(kBlock), 0, st, Vb, ncol, x, dim, part);
      hipLaunchKernelGGL(k_vdot_fin<VC>, dim3(ncol), dim3(kBlock), 0, st, part, G, h, coef, pass,
                         (const double*)nullptr, (const double*)nullptr);
      hipLaunchKernelGGL(k_vaxpy<VC>, dim3(G), dim3(kBlock), 0, st, Vb, ncol, h, x, dim,
                         pass == 1 ? npart : nullptr);
    }
    hipLaunchKernelGGL(k_trl_coef, dim3(1), dim3(kBlock), 0, st, npart, G, coef, jn >= 0 ? jn : m,
                       jn >= 0 ? alpha : nullptr, beta, jn >= 0 ? shifted : 0, jc);  // beta[m]: scratch slot
    if (out && jn >= 0)
      hipLaunchKernelGGL(k_scale_into<VC>, dim3(grid_for(dim)), dim3(kBlock), 0, st, x, out, beta + jn, dim);
    return ED_OK;
  }
  // V[:, k0:k0+nout] = V[:, k0:k0+ncol] Y (Y on the device, ld ncol): in
  // place up to 32 columns, else through Xb and a copy back
  int rotate(int k0, int ncol, int nout, int g) {
    const dim3 gr(std::min(g, 2048));
    if (ncol <= 16)
      hipLaunchKernelGGL((k_rotate_ip<VC, 16>), gr, dim3(kBlock), 0, st, col(Vb, k0), ncol, Y, ncol, nout, dim);
    else if (ncol <= 32 && (!VC || ncol <= 24))
      hipLaunchKernelGGL((k_rotate_ip<VC, VC ? 24 : 32>), gr, dim3(kBlock), 0, st, col(Vb, k0), ncol, Y, ncol,
                         nout, dim);
    else {
      if (!Xb) CK(alloc((void**)&Xb, (size_t)mcap * dim * sizeof(V)));  // first use (nout < mcap)
      hipLaunchKernelGGL(k_rotate<VC>, gr, dim3(kBlock), (size_t)ncol * nout * sizeof(double), st, col(Vb, k0),
                         ncol, Y, ncol, nout, Xb, dim);
      HIPCK(hipMemcpyAsync(col(Vb, k0), Xb, (size_t)nout * dim * sizeof(V), hipMemcpyDeviceToDevice, st));
    }
    HIPCK(hipGetLastError());
    return ED_OK;
  }
  // Lanczos step j: w = H V_j, CGS2, alpha_j, beta_j; V_{j+1} = w / beta_j.
  // Past the sweep's first column (j > j0) the H·v applies the shifted
  // three-term recurrence (EpiTrlLoc) so that the DGKS test can skip the
  // second Gram-Schmidt pass; the first column after a restart couples to
  // every kept Ritz vector and takes the plain product.
  bool local = true;  // false (ED_OPT_TRLAN_NOLOCAL): plain w = H V_j every step (A/B)
  int step(int j, int j0) {
    nhv++;
    const bool loc = local && j > j0;
    // small packed stored sectors, real vectors: the whole step in one workgroup
    if constexpr (!VC) {
      if (solo && fused && path == 0 && s->d_words && !s->hc && s->row0 == 0 && s->nrows == dim &&
          dim <= kOrthSoloMaxDim && j + 1 <= 32) {
        StepSoloArgs a;
        a.diag = (const double*)s->d_diag;
        a.sptr = s->d_sptr;
        a.words = s->d_words;
        a.dict = (const double*)s->d_pdict;
        a.Vb = (const double*)Vb;
        a.x = (double*)w;
        a.out = j + 1 < m ? (double*)col(Vb, j + 1) : nullptr;
        a.coef = coef;
        a.alpha = alpha;
        a.beta = beta;
        a.dim = dim;
        a.j = j;
        a.shifted = loc ? 1 : 0;
        a.locupd = locupd ? 1 : 0;
        const int nc = (j + 1 + 7) / 8 * 8;
        if (nc <= 8) hipLaunchKernelGGL(k_step_solo<8>, dim3(1), dim3(kOrthSoloBlock), 0, st, a);
        else if (nc <= 16) hipLaunchKernelGGL(k_step_solo<16>, dim3(1), dim3(kOrthSoloBlock), 0, st, a);
        else if (nc <= 24) hipLaunchKernelGGL(k_step_solo<24>, dim3(1), dim3(kOrthSoloBlock), 0, st, a);
        else hipLaunchKernelGGL(k_step_solo<32>, dim3(1), dim3(kOrthSoloBlock), 0, st, a);
        HIPCK(hipGetLastError());
        return ED_OK;
      }
    }
    if (loc) {
      EpiTrlLoc<VC> e{w, col(Vb, j - 1), alpha + (j - 1), beta + (j - 1)};
      CK(launch_hxv<VC>(s, path, col(Vb, j), e, st));
    } else {
      EpiStore<VC> e{w};
      CK(launch_hxv<VC>(s, path, col(Vb, j), e, st));
    }
    CK(orth(j + 1, w, j, j + 1 < m ? col(Vb, j + 1) : nullptr, loc ? 1 : 0));
    return ED_OK;
  }
  int sweep(int j0) {
    const int n = m - j0;
    hipGraphExec_t ge = nullptr;
    for (auto& g : graphs)
      if (g.first == j0) ge = g.second;
    if (!ge && n > 2 && graphs_on) {
      hipGraph_t g;
      HIPCK(hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal));
      int rc = ED_OK;
      for (int j = j0; j < m && rc == ED_OK; j++) rc = step(j, j0);
      hipError_t e2 = hipStreamEndCapture(st, &g);
      if (rc != ED_OK) return rc;
      HIPCK(e2);
      HIPCK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
      (void)hipGraphDestroy(g);
      graphs.emplace_back(j0, ge);
      nhv -= n;  // capture does not run anything
    }
    if (ge) {
      HIPCK(hipGraphLaunch(ge, st));
      nhv += n;
    } else {
      for (int j = j0; j < m; j++) CK(step(j, j0));
    }
    HIPCK(hipGetLastError());
    return ED_OK;
  }
};

// Pinned host staging of the per-restart copies (alpha/beta down, the
// projected eigenvectors up): pageable copies go through the runtime's
// staging buffer, a CPU copy and an extra wait each, three per restart.  One
// buffer per host thread, allocated on first use and kept (a farm worker
// reuses it for every sector; freeing pinned memory can synchronise the
// device under the other workers' streams).
static constexpr int kPinnedDoubles = 2 * (64 + 8) + 64 * 64 + 16;
static double* trlan_pinned() {
  static thread_local double* buf = nullptr;
  if (!buf && hipHostMalloc((void**)&buf, kPinnedDoubles * sizeof(double), hipHostMallocDefault) != hipSuccess)
    buf = nullptr;
  return buf;
}

// blocks of the O(dim) Krylov sweeps
// (1024 until round 4: 512 measured 13 % faster per large-sector solve,
// tools/trlan_ab.py --grid; round 6 in the 8-worker farm: 128 and 256 within
// noise of 512, gpurun_out r6j; at the closing build — the medium sectors in
// the lockstep batch, the local-only CGS pass — 256 with the coefficient
// fold at 256 blocks (5 launches per step instead of 7): farm median 0.618
// -> 0.567 s over 6 reps each, lone (6,6) 82-84 -> 85 us per step, 128:
// 0.588 s, gpurun_out r6gc, profiles/r6/grid_cap_ab.json)
static constexpr int kTrlanGridCap = 256;
// ... except the largest sectors (configs[3]'s nine of 627,264-853,776 rows),
// whose lone solve is the critical path of a many-GPU farm: 512 blocks, the
// coefficient sums in their own launches (lone (6,6) 86.5-87.3 -> 83.6-84.2
// us per step, farm median 0.578 -> 0.570 s, gpurun_out r6big,
// profiles/r6/grid_big_ab.json)
static constexpr int64_t kTrlanBigDim = 600000;
// One thick-restart Lanczos solve on the columns [k0, m) of the basis; the
// columns [0, k0) are locked (deflation: every new vector is orthogonalised
// against them, their coefficients are not part of the projected matrix).
// Start vector: v0 (host) if given, else a hash vector from `seed`.  Returns
// the ma = m - k0 Ritz values (ascending) and the ma x ma rotation Z.
template <bool VC>
static int trlan_core(Trlan<VC>& T, int k0, int nev, int maxit, double tol, const void* v0, uint64_t seed,
                      std::vector<double>& theta, std::vector<double>& Z, int* conv_out) {
  using V = val_t<VC>;
  const int m = T.m, ma = m - k0;
  const int64_t dim = T.dim;
  hipStream_t st = T.st;
  const int g = grid_for(dim);
  const int64_t nd = dim * (VC ? 2 : 1);
  const size_t vs = sizeof(V);
  // V_k0 = v0 / |v0| (orthogonal to the locked columns)
  if (v0) HIPCK(hipMemcpyAsync(T.w, v0, dim * vs, hipMemcpyHostToDevice, st));
  else if (seed == 0) hipLaunchKernelGGL(k_default_start, dim3(grid_for(nd)), dim3(kBlock), 0, st, (double*)T.w, nd);
  else hipLaunchKernelGGL(k_hash_vec, dim3(grid_for(nd)), dim3(kBlock), 0, st, (double*)T.w, nd, seed);
  CK(T.orth(k0, T.w, -1));  // CGS2 against the locked columns; the norm -> beta[m]
  double* const hp = T.hp;  // pinned: [0, 72) alpha, [72, 144) beta, [144, ...) Z, last: scalars
  double* const hal = hp;
  double* const hbe = hp + 72;
  double* const hZ = hp + 144;
  double* const hs = hp + kPinnedDoubles - 8;
  HIPCK(hipMemcpyAsync(hs, T.beta + m, sizeof(double), hipMemcpyDeviceToHost, st));
  HIPCK(hipStreamSynchronize(st));
  const double b0 = hs[0];
  if (!(b0 > 0.0)) return fail(ED_ERR_ARG, "zero start vector");
  hipLaunchKernelGGL(k_scale_into<VC>, dim3(g), dim3(kBlock), 0, st, T.w, T.col(T.Vb, k0), T.beta + m, dim);

  std::vector<double> Tm((size_t)ma * ma, 0.0), al(m), be(m);
  auto tm = [&](int i, int j) -> double& { return Tm[i + (size_t)ma * j]; };
  int jstart = k0, conv = 0;
  uint64_t rseed = seed * 7919 + 1;
  for (int it = 0; it < maxit; it++) {
    int j0 = jstart;
    for (;;) {  // expansion j0..m-1, restarted past an invariant subspace
      CK(T.sweep(j0));
      if (T.beta == T.alpha + (hbe - hal)) {
        HIPCK(hipMemcpyAsync(hal, T.alpha, ((hbe - hal) + m) * sizeof(double), hipMemcpyDeviceToHost, st));
      } else {
        HIPCK(hipMemcpyAsync(hal, T.alpha, m * sizeof(double), hipMemcpyDeviceToHost, st));
        HIPCK(hipMemcpyAsync(hbe, T.beta, m * sizeof(double), hipMemcpyDeviceToHost, st));
      }
      HIPCK(hipStreamSynchronize(st));
      std::copy(hal, hal + m, al.begin());
      std::copy(hbe, hbe + m, be.begin());
      int jb = -1;
      for (int j = j0; j < m; j++) {
        const int l = j - k0;
        tm(l, l) = al[j];
        if (l + 1 < ma) tm(l, l + 1) = tm(l + 1, l) = be[j];
        const double scale = fabs(al[j]) + (l > 0 ? fabs(tm(l - 1, l)) : 0.0) + 1e-300;
        if (l + 1 < ma && be[j] < 1e-13 * scale) {
          jb = j;
          break;
        }
      }
      if (jb < 0) break;
      // invariant subspace at jb: continue from a random direction orthogonal to V
      tm(jb - k0, jb - k0 + 1) = tm(jb - k0 + 1, jb - k0) = 0.0;
      hipLaunchKernelGGL(k_hash_vec, dim3(grid_for(nd)), dim3(kBlock), 0, st, (double*)T.w, nd, rseed++);
      CK(T.orth(jb + 1, T.w, -1));
      hipLaunchKernelGGL(k_scale_into<VC>, dim3(g), dim3(kBlock), 0, st, T.w, T.col(T.Vb, jb + 1),
                         T.beta + m, dim);
      HIPCK(hipGetLastError());
      j0 = jb + 1;
      if (j0 >= m) break;
    }
    const double beta = be[m - 1];
    sym_eigh(ma, Tm, theta, Z);
    // ARPACK-style test: |beta_m * Z(m-1,i)| <= tol * max(eps^(2/3), |theta_i|)
    const double eps23 = 3.6e-11;
    conv = 0;
    for (int i = 0; i < nev; i++)
      if (fabs(beta * Z[(ma - 1) + (size_t)ma * i]) <= tol * std::max(eps23, fabs(theta[i]))) conv++;
    if (conv == nev || it == maxit - 1 || m == dim) break;
    // thick restart: keep nkeep Ritz vectors + the residual direction
    // (kept beyond nev: (ma - nev) / 2 — within 5 % of the best of 16
    // restart-length variants on configs[3])
    const int nkeep = std::max(nev, std::min(ma - 2, nev + (ma - nev) / 2));
    // (the previous restart's upload of hZ completed at this sweep's sync)
    std::copy(Z.begin(), Z.begin() + (size_t)ma * ma, hZ);
    HIPCK(hipMemcpyAsync(T.Y, hZ, (size_t)ma * ma * sizeof(double), hipMemcpyHostToDevice, st));
    CK(T.rotate(k0, ma, nkeep, g));
    hipLaunchKernelGGL(k_scale_into<VC>, dim3(g), dim3(kBlock), 0, st, T.w, T.col(T.Vb, k0 + nkeep),
                       T.beta + (m - 1), dim);
    HIPCK(hipGetLastError());
    std::fill(Tm.begin(), Tm.end(), 0.0);
    for (int i = 0; i < nkeep; i++) {
      tm(i, i) = theta[i];
      tm(i, nkeep) = tm(nkeep, i) = beta * Z[(ma - 1) + (size_t)ma * i];
    }
    jstart = k0 + nkeep;
  }
  *conv_out = conv;
  return ED_OK;
}

// Screening solve of the degeneracy probe (trlan_run): is there an
// eigenvalue of H below `cut` on the orthogonal complement of the locked
// columns [0, k0)?  A plain Lanczos recurrence from a hash start vector,
// without restarts and without keeping the Krylov basis: a rolling window of
// two columns (k0, k0+1) behind the locked ones holds v_{k-1} and v_k, and
// every step is orthogonalised against the locked columns and the window by
// the fused CGS (local-only when the locked coefficients are noise) — so a
// step streams k0 + 2 columns, not the k0 + 20 of the thick-restart probe,
// and the Krylov dimension is not capped by a restart.  Every kScreenChunk
// steps the host forms the lowest Ritz value theta of the tridiagonal and
// its residual bound |beta_k s_k| (first-row QL of the reversed matrix,
// ed_tridiag_poles).  *below = 1: theta < cut — a certificate, since every
// Ritz value is a Rayleigh quotient and so >= the complement's lowest
// eigenvalue (the thick-restart probe then finds its vector); 0: theta
// converged to `tol` AND its whole residual interval [theta - r, theta + r]
// above the cut (none); -1: undecided within maxsteps (thick-restart probe).
// Round 5 also decided "none" on the interval alone after 30 steps; that only
// places the eigenvalue nearest theta, not the complement's lowest (an
// unconverged Ritz vector can carry little of a lower eigenvector), so round 6
// requires both.  The interval test matters on its own too: a missed copy just
// under the cut next to a well-converged theta just above it (r ~ tol|theta|
// > theta - lambda_min) fails the interval test and the run goes on until
// theta itself drops below the cut (tests/test_gpu_eigh.py adversarial case).
constexpr int kScreenChunk = 10;
constexpr int kScreenMaxSteps = 400;
constexpr double kProbeMargin = 1e-11;
// hint: column k0 holds the next Ritz vector of the main solve (round 0 of
// the probe) — the start vector is then the hash vector plus that Ritz
// vector at equal norm.  Where nothing was missed the complement's lowest
// eigenvector is the next one, which the mixed start already carries with
// weight ~1/2, so theta converges in fewer steps; a missed copy lies outside
// the main solve's Krylov space (in exact arithmetic) and is reached through
// the hash part, whose overlap with it is 1/sqrt(2) of a pure hash start's.
template <bool VC>
static int probe_screen(Trlan<VC>& T, int k0, int maxsteps, double tol, double cut, uint64_t seed, int* below,
                        bool hint = false) {
  using V = val_t<VC>;
  const int64_t dim = T.dim;
  hipStream_t st = T.st;
  const int64_t nd = dim * (VC ? 2 : 1);
  const int ca = k0, cb = k0 + 1;
  *below = -1;
  if (maxsteps < 2 || k0 + 2 > T.mcap) return ED_OK;
  // the recurrence's alpha/beta in T.alpha/T.beta's place for the duration
  double *pa = nullptr, *pb = nullptr;
  const int na = std::max(maxsteps, T.m) + 2;
  CK(T.alloc((void**)&pa, na * sizeof(double)));
  CK(T.alloc((void**)&pb, na * sizeof(double)));
  double* const sa = T.alpha;
  double* const sb = T.beta;
  struct Restore {
    Trlan<VC>& t; double* a; double* b;
    ~Restore() { t.alpha = a; t.beta = b; }
  } restore{T, sa, sb};
  T.alpha = pa;
  T.beta = pb;
  HIPCK(hipMemsetAsync(T.col(T.Vb, cb), 0, dim * sizeof(V), st));  // v_{-1} = 0
  hipLaunchKernelGGL(k_hash_vec, dim3(grid_for(nd)), dim3(kBlock), 0, st, (double*)T.w, nd, seed);
  if (hint)  // |hash|^2 ~ nd / 3 (uniform in [-1, 1)); the Ritz vector has unit norm
    hipLaunchKernelGGL(k_mix_hint, dim3(grid_for(nd)), dim3(kBlock), 0, st, (double*)T.w,
                       (const double*)T.col(T.Vb, ca), nd, sqrt((double)nd / 3.0));
  CK(T.orth(k0, T.w, -1));  // against the locked columns; the norm -> beta[m]
  hipLaunchKernelGGL(k_scale_into<VC>, dim3(grid_for(dim)), dim3(kBlock), 0, st, T.w, T.col(T.Vb, ca),
                     T.beta + T.m, dim);
  HIPCK(hipGetLastError());
  double* const hp = T.hp;  // pinned staging: alpha | beta of one chunk
  std::vector<double> al, be;
  for (int k0s = 0; k0s < maxsteps; k0s += kScreenChunk) {
    const int k1 = std::min(maxsteps, k0s + kScreenChunk);
    for (int k = k0s; k < k1; k++) {
      const int cur = (k & 1) ? cb : ca, prv = (k & 1) ? ca : cb;
      T.nhv++;
      if (k == 0) {
        EpiStore<VC> e{T.w};
        CK(launch_hxv<VC>(T.s, T.path, T.col(T.Vb, cur), e, st));
      } else {
        EpiTrlLoc<VC> e{T.w, T.col(T.Vb, prv), pa + (k - 1), pb + (k - 1)};
        CK(launch_hxv<VC>(T.s, T.path, T.col(T.Vb, cur), e, st));
      }
      // alpha slot k, basis column cur; v_{k+1} = w / beta_k -> the window's other column
      CK(T.orth(k0 + 2, T.w, k, T.col(T.Vb, prv), k > 0 ? 1 : 0, cur));
    }
    const int n = k1 - k0s;
    HIPCK(hipMemcpyAsync(hp, pa + k0s, n * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(hp + 72, pb + k0s, n * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    al.insert(al.end(), hp, hp + n);
    be.insert(be.end(), hp + 72, hp + 72 + n);
    // lowest Ritz value and the last component of its vector: the reversed
    // tridiagonal's first components
    const int K = (int)al.size();
    std::vector<double> ar(K), br(K, 0.0), E(K), z2(K), z1(K);
    for (int i = 0; i < K; i++) ar[i] = al[K - 1 - i];
    for (int i = 1; i < K; i++) br[i] = be[K - 1 - i];
    if (ed_tridiag_poles(K, ar.data(), br.data(), E.data(), z2.data(), z1.data()) != ED_OK) return ED_OK;
    const double theta = E[0], resid = fabs(be[K - 1] * z1[0]);
    if (theta < cut) {
      *below = 1;
      return ED_OK;
    }
    // invariant Krylov space: theta is an exact eigenvalue of the complement
    // restricted to it (the hash start vector reaches every eigenvector)
    const bool invariant = be[K - 1] < 1e-13 * (fabs(theta) + 1e-300);
    const bool converged = resid <= tol * std::max(3.6e-11, fabs(theta));
    if (invariant || (converged && theta - resid > cut)) {
      *below = 0;
      return ED_OK;
    }
  }
  return ED_OK;
}

// sp_eigh replacement.  A single-vector Krylov method (ARPACK as much as this
// one) sees one direction of each degenerate eigenspace — the other copies
// only through rounding — so the lowest nev of a degenerate spectrum can come
// back with copies missing (configs[3] with the flat bath: 77 of 169
// sectors).  After the solve, the found vectors are locked and the lowest
// eigenvalue of H on their orthogonal complement is computed from a fresh
// random start (deflated solve); when it lies below the current nev-th value
// it is a missed eigenvalue and replaces it; repeated until a deflated solve
// finds nothing lower (ED_OPT_EIGH_NO_VERIFY skips this, A/B).
template <bool VC>
static int trlan_run(ed_sector* s, int nev, int ncv, int maxit, double tol, const void* v0,
                     double* evals, void* evecs, int32_t* nconv, int32_t* nhv) {
  using V = val_t<VC>;
  Trlan<VC> T;
  T.s = s;
  T.path = resolve_path(s, -1);
  T.st = s->stream;
  T.dim = s->dim;
  T.G = (int)std::min<int64_t>(grid_for(s->dim), s->dim > kTrlanBigDim ? 2 * kTrlanGridCap : kTrlanGridCap);
  T.hp = trlan_pinned();
  if (!T.hp) return fail(ED_ERR_OOM, "pinned host staging buffer");
  T.fused = !(s->opts & ED_OPT_TRLAN_UNFUSED);
  if (s->opts & ED_OPT_TRLAN_NOFOLD) T.kFinFoldG = 0;
  T.graphs_on = !(s->opts & ED_OPT_NO_GRAPH);
  T.local = !(s->opts & ED_OPT_TRLAN_NOLOCAL);
  T.solo = !(s->opts & ED_OPT_TRLAN_NOSOLO);
  T.locupd = !(s->opts & ED_OPT_TRLAN_FULLUPD);
  const int64_t dim = s->dim;
  const int m = (int)std::min<int64_t>(ncv, dim);
  if (nev < 1 || nev >= m) return fail(ED_ERR_ARG, "need 1 <= nev < min(ncv, dim)");
  // deflated solves: nev locked columns + mp active ones, within the 64
  // columns the coefficient buffers hold (h/coef/part/alpha/beta below)
  constexpr int kProbeNcv = 20;
  const int mp = (int)std::min<int64_t>(std::min(std::min(m, kProbeNcv), kTrlanMaxCols - nev), dim - nev);
  const bool verify = !(s->opts & ED_OPT_EIGH_NO_VERIFY) && dim > (int64_t)nev + 2 && mp >= 3;
  const int mcap = verify ? std::max(m, nev + mp) : m;
  T.mcap = mcap;
  const size_t vs = sizeof(V);
  CK(T.alloc((void**)&T.Vb, (size_t)mcap * dim * vs));
  CK(T.alloc((void**)&T.w, dim * vs));
  CK(T.alloc((void**)&T.h, kTrlanMaxCols * sizeof(double2)));
  CK(T.alloc((void**)&T.coef, kTrlanMaxCols * sizeof(double2)));
  CK(T.alloc((void**)&T.part, (size_t)kTrlanMaxCols * T.G * sizeof(double2)));
  CK(T.alloc((void**)&T.part2, (size_t)kTrlanMaxCols * T.G * sizeof(double2)));
  CK(T.alloc((void**)&T.npart, (size_t)T.G * sizeof(double)));
  CK(T.alloc((void**)&T.npA, (size_t)T.G * sizeof(double)));
  CK(T.alloc((void**)&T.npB, (size_t)T.G * sizeof(double)));
  CK(T.alloc((void**)&T.lof, sizeof(int)));
  // alpha | beta in one block laid out as the pinned staging (72 apart): one
  // copy down per restart
  CK(T.alloc((void**)&T.alpha, 2 * (kTrlanMaxCols + 8) * sizeof(double)));
  T.beta = T.alpha + (kTrlanMaxCols + 8);
  CK(T.alloc((void**)&T.Y, (size_t)mcap * mcap * sizeof(double)));
  hipStream_t st = T.st;
  const int g = grid_for(dim);
  T.m = m;
  std::vector<double> theta, Z;
  int conv = 0;
  CK(trlan_core(T, 0, nev, maxit, tol, v0, 0, theta, Z, &conv));
  // Ritz vectors -> Vb[0, nev): the result vectors live there from here on
  // (locked columns of the deflated solves); with the probe also the next
  // Ritz vector -> Vb[nev] (the screen's start hint)
  std::copy(Z.begin(), Z.begin() + (size_t)m * m, T.hp + 144);
  HIPCK(hipMemcpyAsync(T.Y, T.hp + 144, (size_t)m * m * sizeof(double), hipMemcpyHostToDevice, st));
  const bool hint = verify && conv == nev && nev + 1 < m && !(s->opts & ED_OPT_EIGH_NOHINT);
  CK(T.rotate(0, m, hint ? nev + 1 : nev, g));
  std::vector<double> ev(theta.begin(), theta.begin() + nev);
  if (verify && conv == nev) {
    for (int round = 0; round < nev; round++) {
      // solve for the lowest eigenvalue on the complement of the nev vectors
      for (auto& gr : T.graphs) (void)hipGraphExecDestroy(gr.second);
      T.graphs.clear();  // captured sweeps depend on m
      T.m = nev + mp;
      std::vector<double> th2, Z2;
      int c2 = 0;
      // the screen's "none" needs only a loose tolerance on top of its
      // residual-interval test (Ritz values approach the lowest from above)
      constexpr double kProbeTol = 1e-5;  // 1e-3 misses copies; 1e-4 and 1e-5 find them
      const double tprobe = std::max(tol, kProbeTol);
      // a copy missed within the margin below ev[nev-1] stays missed, so the
      // margin sits under the 1e-10 Ritz-value bar (round 5: 1e-9, which let
      // a pair 3e-10 below the top through; tests/golden/adversarial_probe.json)
      const double cut = ev[nev - 1] - kProbeMargin * std::max(1.0, fabs(ev[nev - 1]));
      if (!(s->opts & ED_OPT_EIGH_FULLPROBE)) {
        // cheap screen first: a plain Lanczos run on the complement decides
        // most sectors (no missed eigenvalue); the thick-restart probe below
        // runs only when it finds one or cannot decide
        int scr = -1;
        CK(probe_screen(T, nev, (int)std::min<int64_t>(dim - nev, kScreenMaxSteps), tprobe, cut, 3000 + round,
                        &scr, hint && round == 0));
        if (scr == 0) break;
      }
      // the thick-restart probe at the full tolerance: its converged Ritz
      // value lies within r^2/gap (r <= tol|theta|) of the complement's lowest
      // eigenvalue, so "th2 >= cut" is decided on an eigenvalue, not on a
      // loosely converged mixture of a near-cut cluster (round 5 ran it at
      // 1e-5 first and re-solved only below the cut)
      CK(trlan_core(T, nev, 1, maxit, tol, nullptr, 1000 + round, th2, Z2, &c2));
      if (!(c2 == 1 && th2[0] < cut)) break;
      const double mu = th2[0];
      // a missed eigenvalue: its Ritz vector -> w, then insert in order
      // (drop the current largest)
      const int ma2 = T.m - nev;
      std::copy(Z2.begin(), Z2.begin() + ma2, T.hp + 144);
      HIPCK(hipMemcpyAsync(T.Y, T.hp + 144, (size_t)ma2 * sizeof(double), hipMemcpyHostToDevice, st));
      hipLaunchKernelGGL(k_rotate<VC>, dim3(std::min(g, 2048)), dim3(kBlock), (size_t)ma2 * sizeof(double), st,
                         T.col(T.Vb, nev), ma2, T.Y, ma2, 1, T.w, dim);
      HIPCK(hipGetLastError());
      int pos = nev - 1;
      while (pos > 0 && ev[pos - 1] > mu) pos--;
      for (int i = nev - 1; i > pos; i--) {
        ev[i] = ev[i - 1];
        HIPCK(hipMemcpyAsync(T.col(T.Vb, i), T.col(T.Vb, i - 1), dim * vs, hipMemcpyDeviceToDevice, st));
      }
      ev[pos] = mu;
      HIPCK(hipMemcpyAsync(T.col(T.Vb, pos), T.w, dim * vs, hipMemcpyDeviceToDevice, st));
    }
  }
  for (int i = 0; i < nev; i++) evals[i] = ev[i];
  // host or device destination (unified addressing): a farm keeps the
  // sector eigenvectors in HBM and copies back only the kept states
  if (evecs) HIPCK(hipMemcpyAsync(evecs, T.Vb, (size_t)nev * dim * vs, hipMemcpyDefault, st));
  HIPCK(hipStreamSynchronize(st));
  if (nconv) *nconv = conv;
  if (nhv) *nhv = T.nhv;
  return ED_OK;
}

// ------------------------------------------- batched small-sector eigh
// ed_sectors_eigh_batch: trlan_run's algorithm for many small stored sectors
// at once (ed_trlbatch.hpp): every restart cycle of every sector still in its
// main solve, and every 10-step chunk of every degeneracy screen, goes into
// one k_trl_batch launch; the host runs trlan_core's / probe_screen's
// decisions per sector on the mailbox values.  A sector the batch cannot
// finish (an invariant Krylov subspace, a screen that finds an eigenvalue
// below the cut or cannot decide, ED_OPT_EIGH_FULLPROBE) or cannot take
// (complex, not stored, beyond kTbMaxDim rows or kTbMaxCols columns) is
// solved afterwards by trlan_run on its own stream, from the same start.
struct TbSec {
  ed_sector* s = nullptr;
  int64_t dim = 0;
  int m = 0, it = 0, j0 = 0, conv = 0, nhv = 0;
  int state = 0;  // 0 main solve, 1 screen, 2 final rotation pending, 3 done, 4 fall back
  std::vector<double> Tm, theta, Z, ev, sal, sbe;
  int maxsteps = 0, sk = 0;
  double cut = 0.0, tprobe = 0.0;
  bool hint = false;
  TrlTask task{};
  int ny = 0;  // next launch's rotation: the first ny entries of Z (ld m)
};

static double host_default_start(int64_t r) {  // k_default_start's value
  uint64_t z = (uint64_t)(r + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z = z ^ (z >> 31);
  return (double)(z >> 11) * (1.0 / 9007199254740992.0) * 2.0 - 1.0;
}
static char* tb_pinned(size_t n) {  // per host thread, grown on demand, kept
  static thread_local char* buf = nullptr;
  static thread_local size_t cap = 0;
  if (n > cap) {
    if (buf) (void)hipHostFree(buf);
    buf = nullptr;
    cap = 0;
    if (hipHostMalloc((void**)&buf, n, hipHostMallocDefault) != hipSuccess) return nullptr;
    cap = n;
  }
  return buf;
}

static bool tb_eligible(const ed_sector* s, int nev, int ncv) {
  const int m = (int)std::min<int64_t>(ncv, s->dim);
  return s && !s->hc && s->nrows == s->dim && s->row0 == 0 && resolve_path(s, -1) == 0 && s->d_sptr &&
         s->d_diag && (s->d_words || (s->d_cols && s->d_vals)) && s->dim <= kTbMaxDim && m <= kTbMaxCols &&
         nev >= 1 && nev < m && nev + 2 <= kTbMaxCols && s->dim > (int64_t)nev + 2 && s->nslice * 64 >= s->dim &&
         // the multi-kernel A/B alternatives keep their own path
         !(s->opts & (ED_OPT_TRLAN_UNFUSED | ED_OPT_TRLAN_NOLOCAL | ED_OPT_TRLAN_NOSOLO));
}

// One sector's host step after a cycle of the batch (ed_trlbatch.hpp) or of
// the lockstep multi-sector solve (ed_trlmulti.hpp), on its mailbox ml
// (alpha [0, 32) | beta [32, 64) | scalar [64]): trlan_core's projected
// eigenproblem, ARPACK convergence test and thick restart, then
// probe_screen's decisions; sets the sector's next task (b.task, b.ny).
static void tb_advance(TbSec& b, const double* ml, int nev, int maxit, double tol) {
  TrlTask& t = b.task;
  const int m = b.m, ma = m;
  b.ny = 0;
  auto tm = [&](int i, int j) -> double& { return b.Tm[i + (size_t)ma * j]; };
  if (b.state == 0) {  // a main sweep [j0, m) ran (trlan_core)
    if (t.op == kTbStart && !(ml[64] > 0.0)) {
      b.state = 4;
      return;
    }
    b.nhv += m - b.j0;
    int jb = -1;
    for (int j = b.j0; j < m; j++) {
      tm(j, j) = ml[j];
      if (j + 1 < ma) tm(j, j + 1) = tm(j + 1, j) = ml[32 + j];
      const double scale = fabs(ml[j]) + (j > 0 ? fabs(tm(j - 1, j)) : 0.0) + 1e-300;
      if (j + 1 < ma && ml[32 + j] < 1e-13 * scale) {
        jb = j;
        break;
      }
    }
    if (jb >= 0) {  // invariant subspace: trlan_run continues from a random direction
      b.state = 4;
      return;
    }
    const double beta = ml[32 + m - 1];
    sym_eigh(ma, b.Tm, b.theta, b.Z);
    const double eps23 = 3.6e-11;
    b.conv = 0;
    for (int i = 0; i < nev; i++)
      if (fabs(beta * b.Z[(ma - 1) + (size_t)ma * i]) <= tol * std::max(eps23, fabs(b.theta[i]))) b.conv++;
    if (b.conv == nev || b.it == maxit - 1 || m == b.dim) {
      b.ev.assign(b.theta.begin(), b.theta.begin() + nev);
      const int mp = (int)std::min<int64_t>(std::min(std::min(m, 20), kTrlanMaxCols - nev), b.dim - nev);
      const bool verify = !(b.s->opts & ED_OPT_EIGH_NO_VERIFY) && mp >= 3 && b.conv == nev;
      if (verify && (b.s->opts & ED_OPT_EIGH_FULLPROBE)) {
        b.state = 4;
        return;
      }
      b.hint = verify && nev + 1 < m && !(b.s->opts & ED_OPT_EIGH_NOHINT);
      const int nrot = b.hint ? nev + 1 : nev;
      t.op = kTbScreen;
      t.ldy = ma;
      t.nrot = nrot;
      b.ny = ma * nrot;
      t.k0s = 0;
      if (verify) {
        b.state = 1;
        b.maxsteps = (int)std::min<int64_t>(b.dim - nev, kScreenMaxSteps);
        b.cut = b.ev[nev - 1] - kProbeMargin * std::max(1.0, fabs(b.ev[nev - 1]));
        b.tprobe = std::max(tol, 1e-5);
        t.k1 = std::min(b.maxsteps, kScreenChunk);
        t.hint = b.hint ? 1 : 0;
        t.seed = 3000;
        b.sk = 0;
        b.sal.clear();
        b.sbe.clear();
      } else {
        b.state = 2;
        t.k1 = 0;
      }
      return;
    }
    // thick restart (trlan_core)
    const int nkeep = std::max(nev, std::min(ma - 2, nev + (ma - nev) / 2));
    t.op = kTbRestart;
    t.ldy = ma;
    t.nrot = nkeep;
    b.ny = ma * nkeep;
    std::fill(b.Tm.begin(), b.Tm.end(), 0.0);
    for (int i = 0; i < nkeep; i++) {
      tm(i, i) = b.theta[i];
      tm(i, nkeep) = tm(nkeep, i) = beta * b.Z[(ma - 1) + (size_t)ma * i];
    }
    b.j0 = nkeep;
    b.it++;
    return;
  }
  if (b.state == 2) {  // the final rotation ran: done
    b.state = 3;
    return;
  }
  // a screen chunk [k0s, k1) ran (probe_screen)
  const int nst = t.k1 - t.k0s;
  b.nhv += nst;
  for (int q = 0; q < nst; q++) {
    b.sal.push_back(ml[q]);
    b.sbe.push_back(ml[32 + q]);
  }
  t.nrot = 0;
  const int K = (int)b.sal.size();
  std::vector<double> ar(K), br(K, 0.0), E(K), z2(K), z1(K);
  for (int i = 0; i < K; i++) ar[i] = b.sal[K - 1 - i];
  for (int i = 1; i < K; i++) br[i] = b.sbe[K - 1 - i];
  int dec = -1;
  if (ed_tridiag_poles(K, ar.data(), br.data(), E.data(), z2.data(), z1.data()) == ED_OK) {
    const double theta = E[0], resid = fabs(b.sbe[K - 1] * z1[0]);
    if (theta < b.cut) dec = 1;
    else {
      const bool invariant = b.sbe[K - 1] < 1e-13 * (fabs(theta) + 1e-300);
      const bool converged = resid <= b.tprobe * std::max(3.6e-11, fabs(theta));
      if (invariant || (converged && theta - resid > b.cut)) dec = 0;
    }
  } else {
    dec = 2;
  }
  if (dec == 0) b.state = 3;
  else if (dec > 0 || t.k1 >= b.maxsteps) b.state = 4;
  else {
    t.k0s = t.k1;
    t.k1 = std::min(b.maxsteps, t.k0s + kScreenChunk);
  }
}

// Fork-join helpers for the batch's per-sector host work (projected
// eigenproblem, screen QL): kept for one ed_sectors_eigh_batch call; the
// calling thread works too.  With dozens of sectors per cycle the host part
// was ~60 % of a batch (profiles/r6/batch_c4_timeline.json).
struct TbPool {
  std::vector<std::thread> th;
  std::mutex mu;
  std::condition_variable cv, cv_done;
  const std::function<void(int)>* fn = nullptr;
  std::atomic<int> next{0};
  int n = 0, gen = 0, busy = 0;
  bool quit = false;
  explicit TbPool(int nt) {
    for (int i = 0; i < nt; i++) th.emplace_back([this] { loop(); });
  }
  ~TbPool() {
    {
      std::lock_guard<std::mutex> g(mu);
      quit = true;
    }
    cv.notify_all();
    for (auto& t : th) t.join();
  }
  void work() {
    for (int i; (i = next.fetch_add(1)) < n;) (*fn)(i);
  }
  void loop() {
    int seen = 0;
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv.wait(lk, [&] { return quit || gen != seen; });
      if (quit) return;
      seen = gen;
      lk.unlock();
      work();
      lk.lock();
      if (--busy == 0) cv_done.notify_one();
    }
  }
  void run(int count, const std::function<void(int)>& f) {
    if (th.empty() || count < 8) {
      for (int i = 0; i < count; i++) f(i);
      return;
    }
    {
      std::lock_guard<std::mutex> g(mu);
      fn = &f;
      n = count;
      next = 0;
      busy = (int)th.size();
      gen++;
    }
    cv.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu);
    cv_done.wait(lk, [&] { return busy == 0; });
  }
};
static constexpr int kTbHostThreads = 3;  // helpers beside the calling thread

static int tb_run(ed_sector* const* secs, const std::vector<int>& which, int nev, int ncv, const int32_t* maxits,
                  double tol, const double* const* v0, double* evals, void* const* evecs, int32_t* nconv,
                  int32_t* nhv, hipStream_t st, std::vector<int>& fallback) {
  std::vector<TbSec> S;
  std::vector<int> idx;
  for (int i : which) {
    if (!tb_eligible(secs[i], nev, ncv)) {
      fallback.push_back(i);
      continue;
    }
    TbSec b;
    b.s = secs[i];
    b.dim = secs[i]->dim;
    b.m = (int)std::min<int64_t>(ncv, b.dim);
    S.push_back(std::move(b));
    idx.push_back(i);
  }
  const int ns = (int)S.size();
  if (ns == 0) return ED_OK;
  // device: per sector Vb (mcap columns) | w | alpha, beta (72 each) | pa, pb
  // | coef | Y; the ws of all sectors contiguous (one start-vector upload),
  // the mailboxes contiguous (one copy down per launch)
  size_t nw = 0, per = 0;
  std::vector<size_t> off(ns), woff(ns);
  for (int k = 0; k < ns; k++) {
    const int mcap = std::max(S[k].m, nev + 2);
    woff[k] = nw;
    nw += (size_t)S[k].dim;
    off[k] = per;
    per += (size_t)mcap * S[k].dim + 2 * 72 + 2 * kTbScreenLen + 2 * kTrlanMaxCols + kTbMaxCols * kTbMaxCols;
  }
  const size_t nmail = (size_t)ns * kTbMail;
  const size_t ytot = (size_t)ns * kTbMaxCols * kTbMaxCols;  // rotations of one launch, packed
  const size_t bytes = (per + nw + nmail + ytot) * sizeof(double) + (size_t)ns * sizeof(TrlTask);
  char* dbase = nullptr;
  HIPCK(hipMallocAsync((void**)&dbase, bytes, st));
  struct Free {
    char* p; hipStream_t s;
    ~Free() { (void)hipFreeAsync(p, s); }
  } free_guard{dbase, st};
  double* const dsec = (double*)dbase;
  double* const dw = dsec + per;
  double* const dmail = dw + nw;
  TrlTask* const dtask = (TrlTask*)(dmail + nmail);
  // pinned: start vectors | mailboxes | tasks + rotations of one launch
  // (the device mirrors the last part: [tasks | rotations packed])
  const size_t hbytes = (nw + nmail + ytot) * sizeof(double) + (size_t)ns * sizeof(TrlTask);
  char* hp = tb_pinned(hbytes);
  if (!hp) return fail(ED_ERR_OOM, "pinned staging (batch eigh)");
  double* const hv0 = (double*)hp;
  double* const hmail = hv0 + nw;
  TrlTask* const htask = (TrlTask*)(hmail + nmail);
  for (int k = 0; k < ns; k++) {
    TbSec& b = S[k];
    const ed_sector* s = b.s;
    double* p = dsec + off[k];
    const int mcap = std::max(b.m, nev + 2);
    TrlTask& t = b.task;
    t.diag = (const double*)s->d_diag;
    t.sptr = s->d_sptr;
    t.words = s->d_words;
    t.dict = (const double*)s->d_pdict;
    t.cols = s->d_cols;
    t.vals = (const double*)s->d_vals;
    t.dim = b.dim;
    t.Vb = p;
    p += (size_t)mcap * b.dim;
    t.alpha = p;
    t.beta = p + 72;
    p += 144;
    t.pa = p;
    t.pb = p + kTbScreenLen;
    p += 2 * kTbScreenLen;
    t.coef = (double2*)p;
    p += 2 * kTrlanMaxCols;
    t.Y = p;
    t.w = dw + woff[k];
    t.mail = dmail + (size_t)k * kTbMail;
    t.m = b.m;
    t.nev = nev;
    t.locupd = !(s->opts & ED_OPT_TRLAN_FULLUPD);
    t.op = kTbStart;
    b.Tm.assign((size_t)b.m * b.m, 0.0);
    const int i = idx[k];
    if (v0 && v0[i]) memcpy(hv0 + woff[k], v0[i], b.dim * sizeof(double));
    else
      for (int64_t r = 0; r < b.dim; r++) hv0[woff[k] + r] = host_default_start(r);
  }
  HIPCK(hipMemcpyAsync(dw, hv0, nw * sizeof(double), hipMemcpyHostToDevice, st));
  static std::once_flag lds_once;
  static hipError_t lds_err = hipSuccess;
  std::call_once(lds_once, [] {
    lds_err = hipFuncSetAttribute((const void*)k_trl_batch<24>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(kTbMaxDim * sizeof(double)));
    if (lds_err == hipSuccess)
      lds_err = hipFuncSetAttribute((const void*)k_trl_batch<32>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                    (int)(kTbMaxDim * sizeof(double)));
  });
  HIPCK(lds_err);
  std::vector<int> act;
  // per-sector host step after a launch (trlan_core's / probe_screen's logic)
  const std::function<void(int)> process = [&](int a) {
    const int k = act[a];
    tb_advance(S[k], hmail + (size_t)k * kTbMail, nev, maxits[idx[k]], tol);
  };
  TbPool pool(ns >= 8 ? kTbHostThreads : 0);
  for (;;) {
    act.clear();
    for (int k = 0; k < ns; k++)
      if (S[k].state <= 2) act.push_back(k);
    if (act.empty()) break;
    // tasks and rotations of this launch (rotations packed, one copy up)
    const int na = (int)act.size();
    double* const hY = (double*)(htask + na);
    const double* const dY = (const double*)(dtask + na);
    size_t yo = 0;
    int64_t maxdim = 0;
    int maxm = 0;
    for (int a = 0; a < na; a++) {
      TbSec& b = S[act[a]];
      TrlTask t = b.task;
      t.nrot = b.ny > 0 ? t.nrot : 0;
      if (b.ny > 0) {
        std::copy(b.Z.begin(), b.Z.begin() + b.ny, hY + yo);
        t.Y = dY + yo;
        yo += b.ny;
      }
      htask[a] = t;
      maxdim = std::max(maxdim, b.dim);
      maxm = std::max(maxm, std::max(b.m, nev + 2));
    }
    HIPCK(hipMemcpyAsync(dtask, htask, na * sizeof(TrlTask) + yo * sizeof(double), hipMemcpyHostToDevice, st));
    if (maxm <= 24)
      hipLaunchKernelGGL(k_trl_batch<24>, dim3((unsigned)na), dim3(kTbBlock), (size_t)maxdim * sizeof(double), st,
                         (const TrlTask*)dtask);
    else
      hipLaunchKernelGGL(k_trl_batch<32>, dim3((unsigned)na), dim3(kTbBlock), (size_t)maxdim * sizeof(double), st,
                         (const TrlTask*)dtask);
    HIPCK(hipGetLastError());
    HIPCK(hipMemcpyAsync(hmail, dmail, nmail * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    pool.run((int)act.size(), process);
  }
  // results; fall-backs re-solved by the caller
  for (int k = 0; k < ns; k++) {
    TbSec& b = S[k];
    const int i = idx[k];
    if (b.state != 3) {
      fallback.push_back(i);
      if (nhv) nhv[i] = b.nhv;
      continue;
    }
    for (int e = 0; e < nev; e++) evals[(size_t)i * nev + e] = b.ev[e];
    if (evecs && evecs[i])
      HIPCK(hipMemcpyAsync(evecs[i], b.task.Vb, (size_t)nev * b.dim * sizeof(double), hipMemcpyDefault, st));
    if (nconv) nconv[i] = b.conv;
    if (nhv) nhv[i] = b.nhv;
  }
  HIPCK(hipStreamSynchronize(st));
  return ED_OK;
}

// ------------------------------------- lockstep multi-sector eigh
// tm_run: trlan_run's algorithm for stored sectors above the one-workgroup
// batch's size, all of them in lockstep (ed_trlmulti.hpp): one cycle = the
// rotations, then S steps of 7 launches each carrying every running sector,
// one mailbox copy down and the per-sector host step (tb_advance) on the
// pool.  Sectors it cannot take or finish go to `fallback`.
static bool tm_eligible(const ed_sector* s, int nev, int ncv) {
  const int m = (int)std::min<int64_t>(ncv, s->dim);
  return s && !s->hc && s->nrows == s->dim && s->row0 == 0 && resolve_path(s, -1) == 0 && s->d_sptr &&
         s->d_diag && s->d_words && s->d_pdict && m <= kTbMaxCols && nev >= 1 && nev < m &&
         nev + 2 <= kTbMaxCols && s->dim > (int64_t)nev + 2 && s->nslice * 64 >= s->dim &&
         !(s->opts & (ED_OPT_TRLAN_UNFUSED | ED_OPT_TRLAN_NOLOCAL | ED_OPT_TRLAN_NOSOLO));
}

static int tm_run(ed_sector* const* secs, const std::vector<int>& which, int nev, int ncv, const int32_t* maxits,
                  double tol, const double* const* v0, double* evals, void* const* evecs, int32_t* nconv,
                  int32_t* nhv, hipStream_t st, std::vector<int>& fallback) {
  const int ns = (int)which.size();
  if (ns == 0) return ED_OK;
  std::vector<TbSec> S(ns);
  std::vector<TmSec> hs(ns);
  std::vector<size_t> off(ns);
  size_t per = 0;
  for (int k = 0; k < ns; k++) {
    ed_sector* s = secs[which[k]];
    TbSec& b = S[k];
    b.s = s;
    b.dim = s->dim;
    b.m = (int)std::min<int64_t>(ncv, b.dim);
    b.Tm.assign((size_t)b.m * b.m, 0.0);
    // (as one sector's sweep alone, at most kTrlanGridCap blocks: every block
    // of the DGKS and local-only decisions sums all G partials; ~2,048 rows
    // per block below that)
    const int G = (int)std::max<int64_t>(
        1, std::min<int64_t>((b.dim + kTmRowsPerBlock - 1) / kTmRowsPerBlock, kTrlanGridCap));
    hs[k].G = G;
    hs[k].Gh = (int)std::min<int64_t>((b.dim + 4 * kBlock - 1) / (4 * kBlock), 4096);  // 4 rows per thread
    const int mcap = std::max(b.m, nev + 2);
    off[k] = per;
    // (every sub-array starts on a 16-byte boundary: the double2 ones need it)
    per += (size_t)mcap * b.dim + 2 + (size_t)b.dim + 2 + 4 * (size_t)kTrlanMaxCols * G +
           (3 * (size_t)G + 1) / 2 * 2 + 4 * kTrlanMaxCols + 2 + 144 + 2 * kTbScreenLen;
    per = (per + 1) & ~(size_t)1;
  }
  const size_t nmail = (size_t)ns * kTbMail;
  const size_t ytot = (size_t)ns * kTbMaxCols * kTbMaxCols;
  const size_t ctab = (size_t)ns * sizeof(TmCyc) + 2 * (ns + 1) * sizeof(int) + 64;
  const size_t bytes = (per + nmail + ytot) * sizeof(double) + (size_t)ns * sizeof(TmSec) + ctab;
  char* dbase = nullptr;
  HIPCK(hipMallocAsync((void**)&dbase, bytes, st));
  struct Free {
    char* p; hipStream_t s;
    ~Free() { (void)hipFreeAsync(p, s); }
  } free_guard{dbase, st};
  double* const dsec = (double*)dbase;
  double* const dmail = dsec + per;
  TmSec* const dtab = (TmSec*)(dmail + nmail);
  char* const dcyc = (char*)(dtab + ns);  // [TmCyc | boffG | boffH | pad | Y packed] of one cycle
  // pinned: start column / mailboxes | cycle table
  const int64_t maxdim = [&] { int64_t d = 0; for (auto& b : S) d = std::max(d, b.dim); return d; }();
  const size_t hbytes = std::max<size_t>(maxdim, nmail) * sizeof(double) + ctab + ytot * sizeof(double);
  char* hp = tb_pinned(hbytes);
  if (!hp) return fail(ED_ERR_OOM, "pinned staging (multi-sector eigh)");
  double* const hmail = (double*)hp;
  char* const hcyc = hp + std::max<size_t>(maxdim, nmail) * sizeof(double);
  for (int k = 0; k < ns; k++) {
    TbSec& b = S[k];
    const ed_sector* s = b.s;
    TmSec& t = hs[k];
    double* p = dsec + off[k];
    const int mcap = std::max(b.m, nev + 2);
    t.diag = (const double*)s->d_diag;
    t.sptr = s->d_sptr;
    t.words = s->d_words;
    t.dict = (const double*)s->d_pdict;
    t.dim = b.dim;
    // (columns at stride dim, as the sweeps index them; each sub-array starts
    // on a 16-byte boundary)
    auto even = [](size_t q) { return (q + 1) & ~(size_t)1; };
    t.Vb = p;
    p += even((size_t)mcap * b.dim);
    t.w = p;
    p += even(b.dim);
    t.part = (double2*)p;
    p += 2 * (size_t)kTrlanMaxCols * t.G;
    t.part2 = (double2*)p;
    p += 2 * (size_t)kTrlanMaxCols * t.G;
    t.npA = p;
    t.npB = p + t.G;
    t.npart = p + 2 * t.G;
    p += (3 * (size_t)t.G + 1) / 2 * 2;
    t.h = (double2*)p;
    t.coef = (double2*)(p + 2 * kTrlanMaxCols);
    p += 4 * kTrlanMaxCols;
    t.lof = (int*)p;
    p += 2;
    t.alpha = p;
    t.beta = p + 72;
    p += 144;
    t.pa = p;
    t.pb = p + kTbScreenLen;
    t.mail = dmail + (size_t)k * kTbMail;
    b.task.m = b.m;
    b.task.nev = nev;
    b.task.locupd = !(s->opts & ED_OPT_TRLAN_FULLUPD);
    b.task.op = kTbStart;
    // V_0 = v0 / |v0| (host norm)
    double* h0 = (double*)hp;
    const int i = which[k];
    double n2 = 0.0;
    for (int64_t r = 0; r < b.dim; r++) {
      h0[r] = (v0 && v0[i]) ? v0[i][r] : host_default_start(r);
      n2 += h0[r] * h0[r];
    }
    if (!(n2 > 0.0)) {
      b.state = 4;
      continue;
    }
    const double inv = 1.0 / sqrt(n2);
    for (int64_t r = 0; r < b.dim; r++) h0[r] *= inv;
    HIPCK(hipMemcpyAsync(t.Vb, h0, b.dim * sizeof(double), hipMemcpyHostToDevice, st));
    HIPCK(hipStreamSynchronize(st));  // (the staging buffer is reused for the next sector)
  }
  HIPCK(hipMemcpyAsync(dtab, hs.data(), ns * sizeof(TmSec), hipMemcpyHostToDevice, st));
  std::vector<int> act;
  const std::function<void(int)> process = [&](int a) {
    const int k = act[a];
    tb_advance(S[k], hmail + (size_t)k * kTbMail, nev, maxits[which[k]], tol);
  };
  TbPool pool(ns >= 8 ? kTbHostThreads : 0);
  for (;;) {
    act.clear();
    for (int k = 0; k < ns; k++)
      if (S[k].state <= 2) act.push_back(k);
    if (act.empty()) break;
    const int na = (int)act.size();
    TmCyc* const hc = (TmCyc*)hcyc;
    int* const hboG = (int*)(hc + na);
    int* const hboH = hboG + (na + 1);
    const size_t yoff = ((na * sizeof(TmCyc) + 2 * (na + 1) * sizeof(int)) + 63) / 64 * 64;
    double* const hY = (double*)(hcyc + yoff);
    const double* const dY = (const double*)(dcyc + yoff);
    size_t yo = 0;
    int steps = 0, maxm = 0, bG = 0, bH = 0;
    bool rot = false;
    for (int a = 0; a < na; a++) {
      TbSec& b = S[act[a]];
      const TrlTask& t = b.task;
      TmCyc c{};
      c.sec = act[a];
      c.m = b.m;
      c.nev = nev;
      c.locupd = t.locupd;
      c.scale_col = -1;
      c.ldy = t.ldy;
      c.nrot = b.ny > 0 ? t.nrot : 0;
      if (t.op == kTbStart) {
        c.phase = 0;
        c.j0 = 0;
      } else if (t.op == kTbRestart) {
        c.phase = 0;
        c.j0 = t.nrot;
        c.scale_col = t.nrot;
      } else {
        c.phase = 1;
        c.k0s = t.k0s;
        c.k1 = t.k1;
        c.sstart = (t.k0s == 0 && t.k1 > 0) ? 1 : 0;
        c.hint = t.hint;
        c.seed = t.seed;
      }
      if (b.ny > 0) {
        std::copy(b.Z.begin(), b.Z.begin() + b.ny, hY + yo);
        c.Y = dY + yo;
        yo += b.ny;
      }
      rot = rot || c.nrot > 0 || c.scale_col >= 0;
      steps = std::max(steps, c.phase == 0 ? c.m - c.j0 : c.k1 - c.k0s + c.sstart);
      maxm = std::max(maxm, c.phase == 0 ? c.m : nev + 2);
      hc[a] = c;
      hboG[a] = bG;
      hboH[a] = bH;
      bG += hs[act[a]].G;
      bH += hs[act[a]].Gh;
    }
    hboG[na] = bG;
    hboH[na] = bH;
    HIPCK(hipMemcpyAsync(dcyc, hcyc, yoff + yo * sizeof(double), hipMemcpyHostToDevice, st));
    const TmCyc* dc = (const TmCyc*)dcyc;
    const int* dboG = (const int*)(dc + na);
    const int* dboH = dboG + (na + 1);
    if (rot) hipLaunchKernelGGL(k_tm_rotate, dim3(bG), dim3(kBlock), 0, st, dtab, dc, dboG, na);
    for (int q = 0; q < steps; q++) {
      hipLaunchKernelGGL(k_tm_hxv, dim3(bH), dim3(kBlock), 0, st, dtab, dc, dboH, na, q);
      for (int pass = 1; pass <= 3; pass++) {
        if (maxm <= 24) hipLaunchKernelGGL(k_tm_cgs<24>, dim3(bG), dim3(kBlock), 0, st, dtab, dc, dboG, na, q, pass);
        else hipLaunchKernelGGL(k_tm_cgs<32>, dim3(bG), dim3(kBlock), 0, st, dtab, dc, dboG, na, q, pass);
        if (pass < 3)
          hipLaunchKernelGGL(k_tm_fin, dim3(na * kTmFinBlocks), dim3(kBlock), 0, st, dtab, dc, na, q, pass);
      }
      hipLaunchKernelGGL(k_tm_coef, dim3(bG), dim3(kBlock), 0, st, dtab, dc, dboG, na, q);
    }
    hipLaunchKernelGGL(k_tm_mail, dim3(na), dim3(64), 0, st, dtab, dc);
    HIPCK(hipGetLastError());
    HIPCK(hipMemcpyAsync(hmail, dmail, nmail * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCK(hipStreamSynchronize(st));
    pool.run(na, process);
  }
  for (int k = 0; k < ns; k++) {
    TbSec& b = S[k];
    const int i = which[k];
    if (b.state != 3) {
      fallback.push_back(i);
      if (nhv) nhv[i] = b.nhv;
      continue;
    }
    for (int e = 0; e < nev; e++) evals[(size_t)i * nev + e] = b.ev[e];
    if (evecs && evecs[i])
      HIPCK(hipMemcpyAsync(evecs[i], hs[k].Vb, (size_t)nev * b.dim * sizeof(double), hipMemcpyDefault, st));
    if (nconv) nconv[i] = b.conv;
    if (nhv) nhv[i] = b.nhv;
  }
  HIPCK(hipStreamSynchronize(st));
  return ED_OK;
}

template <bool HC, bool VC>
static int kron_split_launch(ed_sector* s, int part, int64_t o, int64_t n, const void* x, void* y, int acc,
                             hipStream_t st) {
  using V = val_t<VC>;
  const int64_t cnt = n * (part == 0 ? s->K.dimup : s->K.dimdw);
  if (cnt == 0) return ED_OK;
  // the two-pass kernels serve the split too (pass U on the row block, pass D
  // on the column strip, ld = nu): same products, same order as
  // k_kron_rows / k_kron_cols
  if (kron2_on(s, 2, VC) && !(s->opts & ED_OPT_SPLIT_SIMPLE)) {
    if (part == 0) return launch_kron_up_any<HC, VC>(s, x, y, st, o, n);
    EpiStore<VC> e{(V*)y};
    return launch_kron_dw<HC, VC>(s, x, acc ? y : nullptr, e, st, (int)n, (int)n);
  }
  if (part == 0)
    hipLaunchKernelGGL((k_kron_rows<HC, VC>), dim3(grid_for(cnt)), dim3(kBlock), 0, st, kron_args<HC>(s), o, n,
                       (const V*)x, (V*)y);
  else
    hipLaunchKernelGGL((k_kron_cols<HC, VC>), dim3(grid_for(cnt)), dim3(kBlock), 0, st, kron_args<HC>(s), n,
                       (const V*)x, (V*)y, acc);
  HIPCK(hipGetLastError());
  return ED_OK;
}

static int kron_split(ed_sector* s, int part, int32_t vtype, int64_t o, int64_t n, const void* x, void* y,
                      int acc, void* stream) {
  if (!s || !x || !y) return fail(ED_ERR_ARG, "null");
  if (!s->kron) return fail(ED_ERR_UNSUPPORTED, "sector has no Kronecker form (normal mode without Jx/Jp, ED_DIRECT)");
  const int64_t lim = part == 0 ? s->K.dimdw : s->K.dimup;
  if (o < 0 || n < 0 || o + n > lim) return fail(ED_ERR_ARG, "row/column range outside the factor dimension");
  if (vtype != 0 && vtype != 1) return fail(ED_ERR_ARG, "vtype must be 0 (real) or 1 (complex)");
  if (vtype == 0 && s->hc) return fail(ED_ERR_ARG, "complex H needs vtype=1");
  HIPCK(hipSetDevice(s->device));
  hipStream_t st = (hipStream_t)stream;
  if (s->hc) return kron_split_launch<true, true>(s, part, o, n, x, y, acc, st);
  return vtype ? kron_split_launch<false, true>(s, part, o, n, x, y, acc, st)
               : kron_split_launch<false, false>(s, part, o, n, x, y, acc, st);
}

// ---------------------------------------------------------------- C-ABI
extern "C" {

const char* ed_gpu_last_error(void) { return ed_err_slot().c_str(); }

// Jz_basis sectors: every off-diagonal element must land inside the sector
// (the reference would insert it at column binary_search(...) = 0).  Host
// pass over the sector with the element generator, before any device build.
struct JzCheckAcc {
  const SectorTables* T;
  bool ok = true;
  void diag(double, double) {}
  void off(uint32_t k, double, double) { ok = ok && table_index(*T, k) >= 0; }
};
static bool jz_conserved(const EdModel& M, const SectorTables& T) {
  JzCheckAcc acc;
  acc.T = &T;
  for (size_t b = 0; b + 1 < T.blk_off.size() && acc.ok; b++) {
    const uint32_t idw = T.blk_idw[b];
    const int32_t c0 = T.cls_start[T.need_cls[idw]];
    for (int64_t r = 0; r < T.blk_off[b + 1] - T.blk_off[b] && acc.ok; r++)
      gen_row(M, T.by_cls[c0 + r] | (idw << T.ns), acc);
  }
  return acc.ok;
}

static int sector_create(const ed_params* p, int32_t q1, int32_t q2, int32_t flags, int64_t row0,
                         int64_t nrows, int32_t device, hipStream_t stream, ed_sector** out) {
  if (!out) return fail(ED_ERR_ARG, "out == NULL");
  *out = nullptr;
  if (!(flags & (ED_STORED | ED_DIRECT))) return fail(ED_ERR_ARG, "flags need ED_STORED or ED_DIRECT");
  int ndev = 0;
  HIPCK(hipGetDeviceCount(&ndev));
  if (device < 0 || device >= ndev) return fail(ED_ERR_ARG, "bad device ordinal");
  HIPCK(hipSetDevice(device));
  ed_sector* s = new ed_sector();
  s->device = device;
  int rc = model_from_params(p, &s->Mh);
  if (rc != ED_OK) {
    delete s;
    return fail(rc, "invalid ed_params (Norb/Nspin/Nbath/ed_mode/bath_type)");
  }
  const bool real_ok = model_is_real(s->Mh);
  if ((flags & ED_REAL) && !real_ok) {
    delete s;
    return fail(ED_ERR_ARG, "ED_REAL requested but impHloc/bath carry imaginary parts");
  }
  s->hc = !(flags & ED_REAL);
  s->flags = flags;
  rc = build_tables(s->Mh.ns, s->Mh.mode, q1, (s->Mh.mode == ED_MODE_NORMAL || s->Mh.jz) ? q2 : 0, &s->T,
                    s->Mh.jz ? s->Mh.lz2 : nullptr);
  if (rc != ED_OK) {
    delete s;
    return fail(rc, "sector tables: bad quantum numbers or dimension beyond int32");
  }
  if (s->T.dim == 0) {
    delete s;
    return fail(ED_ERR_ARG, "empty sector");
  }
  if (s->Mh.jz && !jz_conserved(s->Mh, s->T)) {
    delete s;
    return fail(ED_ERR_UNSUPPORTED,
                "Jz_basis: H moves states out of the (n, twoJz) sector (impHloc / bath / Jp not Jz-conserving)");
  }
  s->dim = s->T.dim;
  if (nrows < 0) {
    row0 = 0;
    nrows = s->dim;
  }
  if (row0 < 0 || nrows < 0 || row0 + nrows > s->dim) {  // nrows == 0: a rank with no rows (dim < MpiSize)
    delete s;
    return fail(ED_ERR_ARG, "row range outside the sector");
  }
  s->row0 = row0;
  s->nrows = nrows;
  s->nslice = (nrows + 63) / 64;
#define TRY(x)            \
  do {                    \
    int r2_ = (x);        \
    if (r2_ != ED_OK) {   \
      sector_free(s);     \
      return r2_;         \
    }                     \
  } while (0)
  // a caller's stream (a farm worker's, reused for every sector it solves)
  // or a private non-blocking one
  hipError_t he = hipSuccess;
  if (stream) {
    s->stream = stream;
    s->own_stream = false;
  } else {
    he = hipStreamCreateWithFlags(&s->stream, hipStreamNonBlocking);
  }
  if (he != hipSuccess) {
    delete s;
    return fail(ED_ERR_HIP, "hipStreamCreate");
  }
  TRY(dalloc_t(s, &s->Md, 1));
  if (dcopy(s, s->Md, &s->Mh, sizeof(EdModel), hipMemcpyHostToDevice) != ED_OK) {
    sector_free(s);
    return fail(ED_ERR_HIP, "model upload");
  }
  TRY(upload(s, &s->d_off, s->T.off));
  TRY(upload(s, &s->d_rank, s->T.rank));
  {
    int64_t* bo;
    uint32_t *bi, *bp;
    int32_t *nn, *ps;
    TRY(upload(s, &bo, s->T.blk_off));
    TRY(upload(s, &bi, s->T.blk_idw));
    TRY(upload(s, &nn, s->T.need_cls));
    TRY(upload(s, &bp, s->T.by_cls));
    TRY(upload(s, &ps, s->T.cls_start));
    TRY(dalloc_t(s, &s->d_map, s->dim));
    hipLaunchKernelGGL(k_build_map, dim3(grid_for(s->dim)), dim3(kBlock), 0, s->stream, bo, bi,
                       (int)s->T.blk_idw.size(), nn, bp, ps, s->T.ns, s->dim, s->d_map);
    if (hipGetLastError() != hipSuccess) {
      sector_free(s);
      return fail(ED_ERR_HIP, "k_build_map launch");
    }
  }
  // Kronecker form: normal mode without Jx/Jp terms (no term moves both spins)
  s->kron = (flags & ED_DIRECT) && s->Mh.mode == ED_MODE_NORMAL && !s->Mh.jhflag && nrows == s->dim;
  if ((flags & ED_STORED) && nrows > 0) TRY(build_stored(s));
  if (s->kron) TRY(build_kron(s));
  // k_direct tables: built here only when the generic matrix-free kernel is
  // the sector's default H·v; otherwise on the first explicit path-1 request
  // (ensure_direct), so stored, Kronecker and GF source sectors keep their
  // build cost and failure modes
  if ((flags & ED_DIRECT) && nrows > 0 && resolve_path(s, -1) == 1) TRY(build_direct(s));
  if (hipStreamSynchronize(s->stream) != hipSuccess) {
    sector_free(s);
    return fail(ED_ERR_HIP, "sector build");
  }
#undef TRY
  *out = s;
  return ED_OK;
}

int ed_sector_create(const ed_params* p, int32_t q1, int32_t q2, int32_t flags, int32_t device,
                     void* stream, ed_sector** out) {
  return sector_create(p, q1, q2, flags, 0, -1, device, (hipStream_t)stream, out);
}

int ed_sector_create_rows(const ed_params* p, int32_t q1, int32_t q2, int32_t flags, int64_t row0,
                          int64_t nrows, int32_t device, void* stream, ed_sector** out) {
  return sector_create(p, q1, q2, flags, row0, nrows, device, (hipStream_t)stream, out);
}

int ed_sector_destroy(ed_sector* s) {
  sector_free(s);
  return ED_OK;
}

// every defined ED_OPT_* bit (include/ed_gpu.h); any other bit is refused
static constexpr int32_t kOptKnown =
    ED_OPT_NO_PERSIST | ED_OPT_PERSIST_STORED | ED_OPT_NO_PREG | ED_OPT_NO_PKRON | ED_OPT_SPLIT_SIMPLE |
    ED_OPT_NO_BATCH | ED_OPT_EIGH_NO_VERIFY | ED_OPT_TRLAN_UNFUSED | ED_OPT_TRLAN_NOFOLD | ED_OPT_NO_GRAPH |
    ED_OPT_TRLAN_NOLOCAL | ED_OPT_TRLAN_NOSOLO | ED_OPT_TRLAN_FULLUPD | ED_OPT_STORED_EXACT |
    ED_OPT_EIGH_FULLPROBE | ED_OPT_NO_FUSED | ED_OPT_EIGH_NOHINT;

int ed_sector_set_options(ed_sector* s, int32_t opts) {
  if (!s) return fail(ED_ERR_ARG, "null");
  if (opts & ~kOptKnown) return fail(ED_ERR_ARG, "unknown ED_OPT_* bits");
  if (opts != s->opts) drop_graph(s);  // a captured recurrence bakes in the kernel choice
  s->opts = opts;
  return ED_OK;
}

int ed_sector_get_info(const ed_sector* s, ed_sector_info* info) {
  if (!s || !info) return fail(ED_ERR_ARG, "null");
  memset(info, 0, sizeof(*info));
  info->dim = s->dim;
  info->row0 = s->row0;
  info->nrows = s->nrows;
  info->nnz = (s->flags & ED_STORED) ? s->nnz : 0;
  info->padded = s->padded;
  info->ns = s->Mh.ns;
  info->mode = s->Mh.mode;
  info->q1 = s->T.q1;
  info->q2 = s->T.q2;
  info->flags = s->flags;
  info->kron = s->kron ? 1 : 0;
  info->dimup = s->T.dimup;
  info->dimdw = s->T.dimdw;
  info->device_bytes = s->bytes;
  info->packed = s->d_words ? 1 : 0;
  info->npdict = s->npdict;
  info->split = s->split ? 1 : 0;
  info->split_far = s->nfar;
  info->split_far_uniform = s->nfar_u;
  info->fused = s->fused ? 1 : 0;
  info->fused_far = s->fu_far;
  info->fused_far_uniform = s->fu_far_u;
  info->fused_bytes = s->fused ? (s->fu_na + s->fu_nl) * 4 + s->fu_nu * 8 + s->nfu * (int64_t)sizeof(FuUnit) : 0;
  info->split_bytes = s->split ? (s->paddedA + s->nlw) * 4 + s->nul * 8 + s->split_meta : 0;
  info->split_list_bytes = s->split ? s->split_listR : 0;
  return ED_OK;
}

int ed_sector_hxv_dev_path(ed_sector* s, int32_t path, int32_t vtype, const void* v, void* hv,
                           void* stream) {
  if (s && s->nrows == 0) return ED_OK;  // no local rows: nothing to write
  if (!s || !v || !hv) return fail(ED_ERR_ARG, "null");
  int pth = resolve_path(s, path);
  if (pth < 0) return fail(ED_ERR_ARG, "H·v path not available for this sector");
  HIPCK(hipSetDevice(s->device));
  CK(ensure_direct(s, pth, (hipStream_t)stream));
  hipStream_t st = (hipStream_t)stream;
  if (vtype == 1) {
    EpiStore<true> e{(double2*)hv};
    return launch_hxv<true>(s, pth, v, e, st);
  }
  if (vtype == 0) {
    EpiStore<false> e{(double*)hv};
    return launch_hxv<false>(s, pth, v, e, st);
  }
  return fail(ED_ERR_ARG, "vtype must be 0 (real) or 1 (complex)");
}

int ed_sector_col_mask(const ed_sector* s, uint32_t* mask_dev, void* stream) {
  if (!s || !mask_dev) return fail(ED_ERR_ARG, "null");
  HIPCK(hipSetDevice(s->device));
  hipStream_t st = (hipStream_t)stream;
  HIPCK(hipMemsetAsync(mask_dev, 0, (size_t)((s->dim + 31) / 32) * 4, st));
  if (s->nrows == 0) return ED_OK;
  DevIndex idx{s->d_off, s->d_rank, s->T.ns, s->T.nst - 1};
  hipLaunchKernelGGL(k_mark_cols, dim3(grid_for(s->nrows)), dim3(kBlock), 0, st, s->Md, s->d_map + s->row0,
                     s->nrows, idx, mask_dev);
  HIPCK(hipGetLastError());
  return ED_OK;
}

int ed_sector_kron_rows(ed_sector* s, int32_t vtype, int64_t w0, int64_t nw, const void* x, void* y,
                        void* stream) {
  return kron_split(s, 0, vtype, w0, nw, x, y, 0, stream);
}

int ed_sector_kron_cols(ed_sector* s, int32_t vtype, int64_t u0, int64_t nu, const void* xt, void* yt,
                        int32_t accumulate, void* stream) {
  return kron_split(s, 1, vtype, u0, nu, xt, yt, accumulate, stream);
}

int ed_sector_hxv_dev(ed_sector* s, int32_t vtype, const void* v, void* hv, void* stream) {
  return ed_sector_hxv_dev_path(s, -1, vtype, v, hv, stream);
}

int ed_sector_hxv(ed_sector* s, int32_t nloc, const double* v, double* hv) {
  if (!s || !v || !hv) return fail(ED_ERR_ARG, "null");
  CK(whole_only(s));
  // directMatVec_cc: "Nloc != dim(isector)" (DIRECT_HxV.f90:50)
  if ((int64_t)nloc != s->dim) return fail(ED_ERR_ARG, "ed_gpu_hxv ERROR: Nloc != dim(isector)");
  HIPCK(hipSetDevice(s->device));
  if (!s->d_x) {
    CK(dalloc(s, &s->d_x, s->dim * 16));
    CK(dalloc(s, &s->d_y, s->dim * 16));
  }
  HIPCK(hipMemcpyAsync(s->d_x, v, s->dim * 16, hipMemcpyHostToDevice, s->stream));
  CK(ed_sector_hxv_dev(s, 1, s->d_x, s->d_y, s->stream));
  HIPCK(hipMemcpyAsync(hv, s->d_y, s->dim * 16, hipMemcpyDeviceToHost, s->stream));
  HIPCK(hipStreamSynchronize(s->stream));
  return ED_OK;
}

int ed_sector_map(const ed_sector* s, uint32_t* map_host) {
  if (!s || !map_host) return fail(ED_ERR_ARG, "null");
  HIPCK(hipSetDevice(s->device));
  CK(dcopy(s, map_host, s->d_map, s->dim * sizeof(uint32_t), hipMemcpyDeviceToHost));
  return ED_OK;
}

int ed_sector_dump_csr(const ed_sector* s, int64_t* rowptr, int32_t* cols, double* vals) {
  if (!s || !rowptr || !cols || !vals) return fail(ED_ERR_ARG, "null");
  if (!(s->flags & ED_STORED)) return fail(ED_ERR_STATE, "sector was built without ED_STORED");
  HIPCK(hipSetDevice(s->device));
  const int64_t dim = s->nrows, ns = s->nslice, slots = s->padded;  // local rows, global columns
  rowptr[0] = 0;
  if (dim == 0) return ED_OK;
  const int hw = s->hc ? 2 : 1;
  std::vector<uint16_t> cnt(dim);
  std::vector<int64_t> sptr(ns + 1);
  std::vector<int32_t> sc(slots);
  std::vector<double> sv(slots * hw), dg(dim * hw);
  CK(dcopy(s, cnt.data(), s->d_cnt, dim * 2, hipMemcpyDeviceToHost));
  CK(dcopy(s, sptr.data(), s->d_sptr, (ns + 1) * 8, hipMemcpyDeviceToHost));
  CK(dcopy(s, sc.data(), s->d_cols, slots * 4, hipMemcpyDeviceToHost));
  CK(dcopy(s, sv.data(), s->d_vals, slots * 8 * hw, hipMemcpyDeviceToHost));
  CK(dcopy(s, dg.data(), s->d_diag, dim * 8 * hw, hipMemcpyDeviceToHost));
  int64_t q = 0;
  rowptr[0] = 0;
  for (int64_t i = 0; i < dim; i++) {
    cols[q] = (int32_t)(s->row0 + i);
    vals[2 * q] = dg[hw * i];
    vals[2 * q + 1] = hw == 2 ? dg[2 * i + 1] : 0.0;
    q++;
    int64_t base = sptr[i >> 6] + (i & 63);
    for (int k = 0; k < cnt[i]; k++) {
      int64_t t = base + 64 * (int64_t)k;
      cols[q] = sc[t];
      vals[2 * q] = sv[hw * t];
      vals[2 * q + 1] = hw == 2 ? sv[2 * t + 1] : 0.0;
      q++;
    }
    rowptr[i + 1] = q;
  }
  return ED_OK;
}

int ed_sector_sell_view(const ed_sector* s, ed_sell_view* v) {
  if (!s || !v) return fail(ED_ERR_ARG, "null");
  if (!(s->flags & ED_STORED)) return fail(ED_ERR_STATE, "sector was built without ED_STORED");
  v->dim = s->dim;
  v->nslice = s->nslice;
  v->slots = s->padded;
  v->value_bytes = s->hc ? 16 : 8;
  v->pad = 0;
  v->diag = s->d_diag;
  v->sptr = s->d_sptr;
  v->cols = s->d_cols;
  v->vals = s->d_vals;
  v->rowcnt = s->d_cnt;
  return ED_OK;
}

// One Lanczos driver for every entry point: persistent one-workgroup kernel
// when the sector fits a CU, graph-captured two-kernel recurrence otherwise.
struct LancDriver {
  ed_sector* s;
  int vc, path, pm;
  bool basis;
  hipStream_t st;
  int start(double thresh) {
    if (pm >= 0) return persist_set_thresh(s, thresh, st);
    return vc ? lanc_start<true>(s, thresh, st) : lanc_start<false>(s, thresh, st);
  }
  int iters(int n, bool first) {
    if (pm >= 0)
      return vc ? persist_iters<true>(s, pm, basis, n, first ? 1 : 0, st)
                : persist_iters<false>(s, pm, basis, n, first ? 1 : 0, st);
    return vc ? lanc_iters<true>(s, path, basis, n, st) : lanc_iters<false>(s, path, basis, n, st);
  }
};

static int make_driver(ed_sector* s, int vtype, bool basis, LancDriver* d) {
  CK(whole_only(s));
  d->s = s;
  d->vc = vtype ? 1 : 0;
  if (d->vc == 0 && s->hc) return fail(ED_ERR_ARG, "complex H needs vtype=1");
  d->path = resolve_path(s, -1);
  d->pm = persist_mode(s, d->vc, d->path);
  d->basis = basis;
  d->st = s->stream;
  return ED_OK;
}

static int lanc_load_start(ed_sector* s, int vc, const void* v0, bool v0_device) {
  const size_t vs = vc ? 16 : 8;
  if (v0) {
    HIPCK(hipMemcpyAsync(s->ws.R, v0, s->dim * vs,
                         v0_device ? hipMemcpyDeviceToDevice : hipMemcpyHostToDevice, s->stream));
  } else {
    hipLaunchKernelGGL(k_default_start, dim3(grid_for(s->dim * (vc ? 2 : 1))), dim3(kBlock), 0,
                       s->stream, (double*)s->ws.R, s->dim * (vc ? 2 : 1));
    HIPCK(hipGetLastError());
  }
  return ED_OK;
}

// Fixed-length run from a device start vector (benchmark entry point).
int ed_sector_lanc_run(ed_sector* s, int32_t vtype, const void* v0_dev, int32_t niter,
                       double* alfa, double* beta, float* ms, void* stream) {
  (void)stream;
  if (!s || niter < 1) return fail(ED_ERR_ARG, "bad args");
  HIPCK(hipSetDevice(s->device));
  LancDriver d;
  CK(make_driver(s, vtype, false, &d));
  CK(lanc_prepare(s, d.vc, niter, false, 0));
  CK(lanc_load_start(s, d.vc, v0_dev, true));
  LancWS& w = s->ws;
  for (hipEvent_t& e : w.ev)
    if (!e) HIPCK(hipEventCreate(&e));
  hipEvent_t e0 = w.ev[0], e1 = w.ev[1];
  int rc = d.start(1e-300);
  if (rc == ED_OK) {
    HIPCK(hipEventRecord(e0, d.st));
    rc = d.iters(niter, true);
    HIPCK(hipEventRecord(e1, d.st));
  }
  // one host sync for the run and one pinned copy of alpha | beta
  const size_t nab = (size_t)w.cap + 2 + niter;
  if (rc == ED_OK && (alfa || beta))
    HIPCK(hipMemcpyAsync(w.h_ab, w.alpha, nab * sizeof(double), hipMemcpyDeviceToHost, d.st));
  HIPCK(hipStreamSynchronize(d.st));
  CK(rc);
  if (alfa) memcpy(alfa, w.h_ab, niter * sizeof(double));
  if (beta) memcpy(beta, w.h_ab + w.cap + 2, niter * sizeof(double));
  if (ms) HIPCK(hipEventElapsedTime(ms, e0, e1));
  return ED_OK;
}

int ed_sector_lanc_tridiag(ed_sector* s, int32_t vtype, const void* v0, int32_t nitermax,
                           double threshold, double* alfa, double* beta, int32_t* nlanc) {
  if (!s || !alfa || !beta || nitermax < 1) return fail(ED_ERR_ARG, "bad args");
  HIPCK(hipSetDevice(s->device));
  LancDriver d;
  CK(make_driver(s, vtype, false, &d));
  CK(lanc_prepare(s, d.vc, nitermax, false, 0));
  CK(lanc_load_start(s, d.vc, v0, false));
  CK(d.start(threshold));
  CK(d.iters(nitermax, true));
  std::vector<double> a(nitermax + 1), b(nitermax + 2);
  HIPCK(hipMemcpyAsync(a.data(), s->ws.alpha, nitermax * 8, hipMemcpyDeviceToHost, d.st));
  HIPCK(hipMemcpyAsync(b.data(), s->ws.beta, (nitermax + 1) * 8, hipMemcpyDeviceToHost, d.st));
  LancState hs;
  HIPCK(hipMemcpyAsync(&hs, s->ws.st, sizeof(hs), hipMemcpyDeviceToHost, d.st));
  HIPCK(hipStreamSynchronize(d.st));
  // lanczos_plain_tridiag_c: alanc(iter)=a; if(iter<nitermax)blanc(iter+1)=b; exit if |b|<thr
  int n = hs.iter;
  for (int q = 0; q < nitermax; q++) {
    alfa[q] = q < n ? a[q] : 0.0;
    beta[q] = (q >= 1 && q <= n) ? b[q] : 0.0;
  }
  beta[0] = 0.0;
  if (nlanc) *nlanc = n;
  return ED_OK;
}

// sp_lanc_tridiag for nseed start vectors on one sector (GF seeds of one
// target sector: ED_GF_NORMAL.f90:180-193, ED_GF_NONSU2.f90:343-886).  When
// the sector runs the persistent one-workgroup recurrence, all seeds go in
// ONE launch, one workgroup each (same per-workgroup code as a single run:
// identical alpha/beta); otherwise the seeds run one after the other.
int ed_sector_lanc_tridiag_batch(ed_sector* s, int32_t vtype, int32_t nseed, const void* v0_dev,
                                 int32_t nitermax, double threshold, double* alfa, double* beta,
                                 int32_t* nlanc) {
  if (!s || !v0_dev || !alfa || !beta || nitermax < 1 || nseed < 1) return fail(ED_ERR_ARG, "bad args");
  HIPCK(hipSetDevice(s->device));
  LancDriver d;
  CK(make_driver(s, vtype, false, &d));
  const size_t vs = d.vc ? 16 : 8;
  auto unpack = [&](int k, const double* a, const double* b, int n) {
    double* al = alfa + (size_t)k * nitermax;
    double* be = beta + (size_t)k * nitermax;
    for (int q = 0; q < nitermax; q++) {
      al[q] = q < n ? a[q] : 0.0;
      be[q] = (q >= 1 && q <= n) ? b[q] : 0.0;
    }
    be[0] = 0.0;
    if (nlanc) nlanc[k] = n;
  };
  if (d.pm < 0 || (s->opts & ED_OPT_NO_BATCH)) {
    CK(lanc_prepare(s, d.vc, nitermax, false, 0));
    for (int k = 0; k < nseed; k++) {
      CK(lanc_load_start(s, d.vc, (const unsigned char*)v0_dev + (size_t)k * s->dim * vs, true));
      CK(d.start(threshold));
      CK(d.iters(nitermax, true));
      std::vector<double> a(nitermax + 1), b(nitermax + 2);
      LancState hs;
      HIPCK(hipMemcpyAsync(a.data(), s->ws.alpha, nitermax * 8, hipMemcpyDeviceToHost, d.st));
      HIPCK(hipMemcpyAsync(b.data(), s->ws.beta, (nitermax + 1) * 8, hipMemcpyDeviceToHost, d.st));
      HIPCK(hipMemcpyAsync(&hs, s->ws.st, sizeof(hs), hipMemcpyDeviceToHost, d.st));
      HIPCK(hipStreamSynchronize(d.st));
      unpack(k, a.data(), b.data(), hs.iter);
    }
    return ED_OK;
  }
  CK(lanc_prepare(s, d.vc, nitermax, false, 0));  // register tables / dictionaries of the persistent mode
  PersistBatch bt;
  bt.nb = nseed;
  bt.ldr = s->dim;
  bt.ldp = (int64_t)p_rows(s);
  bt.ldab = 2 * ((int64_t)nitermax + 2);
  hipStream_t st = d.st;
  void *R = nullptr, *P = nullptr, *ab = nullptr, *sts = nullptr;
  HIPCK(hipMallocAsync(&R, (size_t)nseed * bt.ldr * vs, st));
  HIPCK(hipMallocAsync(&P, (size_t)nseed * bt.ldp * vs, st));
  HIPCK(hipMallocAsync(&ab, (size_t)nseed * bt.ldab * 8, st));
  HIPCK(hipMallocAsync(&sts, (size_t)nseed * sizeof(LancState), st));
  auto release = [&]() {
    (void)hipFreeAsync(R, st);
    (void)hipFreeAsync(P, st);
    (void)hipFreeAsync(ab, st);
    (void)hipFreeAsync(sts, st);
  };
  bt.R = R;
  bt.P = P;
  bt.st = (LancState*)sts;
  bt.alpha = (double*)ab;
  bt.beta = (double*)ab + nitermax + 2;
  s->pthresh = threshold;
  int rc = ED_OK;
  if (hipMemcpyAsync(R, v0_dev, (size_t)nseed * s->dim * vs, hipMemcpyDeviceToDevice, st) != hipSuccess ||
      hipMemsetAsync(P, 0, (size_t)nseed * bt.ldp * vs, st) != hipSuccess ||
      hipMemsetAsync(ab, 0, (size_t)nseed * bt.ldab * 8, st) != hipSuccess ||
      hipMemsetAsync(sts, 0, (size_t)nseed * sizeof(LancState), st) != hipSuccess)
    rc = fail(ED_ERR_HIP, "batch workspace");
  if (rc == ED_OK)
    rc = d.vc ? persist_iters<true>(s, d.pm, false, nitermax, 1, st, &bt)
              : persist_iters<false>(s, d.pm, false, nitermax, 1, st, &bt);
  std::vector<double> hab((size_t)nseed * bt.ldab);
  std::vector<LancState> hst(nseed);
  if (rc == ED_OK) {
    HIPCK(hipMemcpyAsync(hab.data(), ab, hab.size() * 8, hipMemcpyDeviceToHost, st));
    HIPCK(hipMemcpyAsync(hst.data(), sts, nseed * sizeof(LancState), hipMemcpyDeviceToHost, st));
  }
  release();
  HIPCK(hipStreamSynchronize(st));
  CK(rc);
  for (int k = 0; k < nseed; k++) {
    // a run that never broke down ends with st->iter = nitermax
    const double* a = hab.data() + (size_t)k * bt.ldab;
    unpack(k, a, a + nitermax + 2, hst[k].iter);
  }
  return ED_OK;
}

// dst must be exactly the sector the operator maps src into (getCsector /
// getCDGsector, ED_SETUP.f90:464-495, 590-619, 750-768); otherwise targets
// would fall outside dst's index tables
static int check_op_target(const ed_sector* src, const ed_sector* dst, int32_t op, int32_t level) {
  if (!src || !dst) return fail(ED_ERR_ARG, "null");
  if (src->device != dst->device) return fail(ED_ERR_ARG, "sectors on different devices");
  if (op != 0 && op != 1) return fail(ED_ERR_ARG, "op must be 0 (c) or 1 (c^+)");
  if (level < 0 || level >= 2 * src->Mh.ns || src->Mh.ns != dst->Mh.ns)
    return fail(ED_ERR_ARG, "level outside the 2*Ns Fock levels / mismatched models");
  const int ns = src->Mh.ns, d = op == 1 ? 1 : -1, up = level < ns;
  int e1 = src->T.q1, e2 = src->T.q2;
  if (src->Mh.mode == ED_MODE_NORMAL) {
    if (up) e1 += d; else e2 += d;
  } else if (src->Mh.mode == ED_MODE_SUPERC) {
    e1 += up ? d : -d;
  } else {
    e1 += d;
    // getCsector_Jz / getCDGsector_Jz (ED_SETUP.f90:769-805): twoJz -/+ (2*Lzdiag(iorb) + Szdiag(ispin))
    if (src->Mh.jz) e2 += d * (src->Mh.lz2[up ? level : level - ns] + (up ? 1 : -1));
  }
  if (dst->Mh.mode != src->Mh.mode || dst->Mh.jz != src->Mh.jz || dst->T.q1 != e1 || dst->T.q2 != e2)
    return fail(ED_ERR_ARG, "dst is not the sector reached by the operator");
  return ED_OK;
}

int ed_sector_apply_op(const ed_sector* src, const ed_sector* dst, int32_t op, int32_t level,
                       int32_t vtype, const void* src_vec, void* dst_vec, void* stream) {
  if (!src_vec || !dst_vec) return fail(ED_ERR_ARG, "null");
  CK(check_op_target(src, dst, op, level));
  CK(whole_only(src));
  CK(whole_only(dst));
  HIPCK(hipSetDevice(src->device));
  hipStream_t st = (hipStream_t)stream;
  const size_t vs = vtype ? 16 : 8;
  HIPCK(hipMemsetAsync(dst_vec, 0, dst->dim * vs, st));
  DevIndex idx{dst->d_off, dst->d_rank, dst->T.ns, dst->T.nst - 1};
  if (vtype)
    hipLaunchKernelGGL(k_apply_op<true>, dim3(grid_for(src->dim)), dim3(kBlock), 0, st, src->d_map,
                       src->dim, idx, op, level, (const double2*)src_vec, (double2*)dst_vec);
  else
    hipLaunchKernelGGL(k_apply_op<false>, dim3(grid_for(src->dim)), dim3(kBlock), 0, st, src->d_map,
                       src->dim, idx, op, level, (const double*)src_vec, (double*)dst_vec);
  HIPCK(hipGetLastError());
  return ED_OK;
}

int ed_sector_apply_op_acc(const ed_sector* src, const ed_sector* dst, int32_t op, int32_t level,
                           double coef_re, double coef_im, int32_t vtype, const void* src_vec,
                           void* dst_vec, void* stream) {
  if (!src_vec || !dst_vec) return fail(ED_ERR_ARG, "null");
  if (!vtype && coef_im != 0.0) return fail(ED_ERR_ARG, "complex coefficient needs vtype=1");
  CK(whole_only(src));
  CK(whole_only(dst));
  CK(check_op_target(src, dst, op, level));
  HIPCK(hipSetDevice(src->device));
  hipStream_t st = (hipStream_t)stream;
  DevIndex idx{dst->d_off, dst->d_rank, dst->T.ns, dst->T.nst - 1};
  if (vtype)
    hipLaunchKernelGGL(k_apply_op_acc<true>, dim3(grid_for(src->dim)), dim3(kBlock), 0, st,
                       src->d_map, src->dim, idx, op, level, coef_re, coef_im,
                       (const double2*)src_vec, (double2*)dst_vec);
  else
    hipLaunchKernelGGL(k_apply_op_acc<false>, dim3(grid_for(src->dim)), dim3(kBlock), 0, st,
                       src->d_map, src->dim, idx, op, level, coef_re, coef_im,
                       (const double*)src_vec, (double*)dst_vec);
  HIPCK(hipGetLastError());
  return ED_OK;
}

// Poles of one GF continued fraction: eigenvalues of tridiag(alfa[0:n],
// beta[1:n]) and the squared first components of the eigenvectors, the
// quantities add_to_lanczos_gf_nonsu2 takes from tql2 (ED_GF_NONSU2.f90:936,
// ED_GF_SHARED.f90:76-214; add_to_lanczos_gf_normal uses eigh,
// ED_GF_NORMAL.f90:612-618).  The EISPACK implicit-QL iteration with the
// rotations applied to the first row of Z only (Z starts as the identity, so
// that row starts as e_1): O(n^2) instead of the O(n^3) full eigenvector
// accumulation; same pythag, shifts and convergence test as tql2.
static double ql_pythag(double a, double b) {
  double p = std::max(fabs(a), fabs(b));
  if (p == 0.0) return p;
  double r = std::min(fabs(a), fabs(b)) / p;
  r = r * r;
  for (;;) {
    const double t = 4.0 + r;
    if (t == 4.0) break;
    const double q = r / t, u = 1.0 + 2.0 * q;
    p = u * p;
    const double qu = q / u;
    r = (qu * qu) * r;
  }
  return p;
}

int ed_tridiag_poles(int32_t n, const double* alfa, const double* beta, double* E, double* z2, double* z1) {
  if (n < 1 || !alfa || !beta || !E || !z2) return fail(ED_ERR_ARG, "bad args");
  std::vector<double> e(n, 0.0), z(n, 0.0);
  for (int i = 0; i < n; i++) E[i] = alfa[i];
  for (int i = 0; i + 1 < n; i++) e[i] = beta[i + 1];  // e[i] = T(i, i+1); e[n-1] = 0
  z[0] = 1.0;
  double f = 0.0, tst1 = 0.0;
  for (int l = 0; l < n; l++) {
    tst1 = std::max(tst1, fabs(E[l]) + fabs(e[l]));
    int m = l;
    while (m < n && tst1 + fabs(e[m]) != tst1) m++;
    if (m >= n) m = n - 1;  // e[n-1] == 0 stops the scan at n-1
    if (m != l) {
      for (int it = 0;; it++) {
        if (it >= 30) return fail(ED_ERR_NOCONV, "tridiagonal QL: no convergence");
        const double g0 = E[l];
        double p = (E[l + 1] - g0) / (2.0 * e[l]);
        double r = ql_pythag(p, 1.0);
        const double sr = p >= 0.0 ? fabs(r) : -fabs(r);
        E[l] = e[l] / (p + sr);
        E[l + 1] = e[l] * (p + sr);
        const double dl1 = E[l + 1];
        double h = g0 - E[l];
        for (int i = l + 2; i < n; i++) E[i] -= h;
        f += h;
        p = E[m];
        double c = 1.0, c2 = 1.0, c3 = 1.0, s = 0.0, s2 = 0.0;
        const double el1 = e[l + 1];
        for (int i = m - 1; i >= l; i--) {
          c3 = c2;
          c2 = c;
          s2 = s;
          const double g = c * e[i];
          h = c * p;
          r = ql_pythag(p, e[i]);
          e[i + 1] = s * r;
          s = e[i] / r;
          c = p / r;
          p = c * E[i] - s * g;
          E[i + 1] = h + s * (c * g + s * E[i]);
          const double zh = z[i + 1];  // first row of Z only
          z[i + 1] = s * z[i] + c * zh;
          z[i] = c * z[i] - s * zh;
        }
        p = -s * s2 * c3 * el1 * e[l] / dl1;
        e[l] = s * p;
        E[l] = c * p;
        if (!(tst1 + fabs(e[l]) > tst1)) break;
      }
    }
    E[l] += f;
  }
  // ascending order (selection sort, as tql2)
  for (int i = 0; i + 1 < n; i++) {
    int k = i;
    for (int j = i + 1; j < n; j++)
      if (E[j] < E[k]) k = j;
    if (k != i) {
      std::swap(E[i], E[k]);
      std::swap(z[i], z[k]);
    }
  }
  for (int i = 0; i < n; i++) z2[i] = z[i] * z[i];
  if (z1)
    for (int i = 0; i < n; i++) z1[i] = z[i];
  return ED_OK;
}

int ed_gf_add_poles(int32_t nfrac, const int32_t* npole, const double* E, const double* z, const double* peso_bz,
                    const double* Ei, const int32_t* isign, const int32_t* comp, const double* wm, int32_t lmats,
                    const double* wr, int32_t lreal, double eps, double* gm, double* gr, void* stream) {
  if (nfrac < 0 || lmats < 0 || lreal < 0) return fail(ED_ERR_ARG, "bad sizes");
  if (nfrac == 0 || lmats + lreal == 0) return ED_OK;
  if (!npole || !E || !z || !peso_bz || !Ei || !isign || !comp || (lmats && (!wm || !gm)) ||
      (lreal && (!wr || !gr)))
    return fail(ED_ERR_ARG, "null");
  std::vector<GfFrac> fr(nfrac);
  int64_t np = 0;
  for (int f = 0; f < nfrac; f++) {
    if (npole[f] < 0 || comp[f] < 0 || (isign[f] != 1 && isign[f] != -1)) return fail(ED_ERR_ARG, "bad fraction");
    fr[f].p0 = (int32_t)np;
    fr[f].np = npole[f];
    fr[f].comp = comp[f];
    fr[f].isign = isign[f];
    fr[f].pr = peso_bz[2 * f];
    fr[f].pi = peso_bz[2 * f + 1];
    fr[f].ei = Ei[f];
    fr[f].pad = 0.0;
    np += npole[f];
  }
  // one staging buffer: fractions | E | z
  const size_t bf = fr.size() * sizeof(GfFrac), be = (size_t)std::max<int64_t>(np, 1) * 8;
  std::vector<unsigned char> hb(bf + 2 * be);
  memcpy(hb.data(), fr.data(), bf);
  if (np) {
    memcpy(hb.data() + bf, E, np * 8);
    memcpy(hb.data() + bf + be, z, np * 8);
  }
  hipStream_t st = (hipStream_t)stream;
  void* d = nullptr;
  HIPCK(hipMallocAsync(&d, hb.size(), st));
  HIPCK(hipMemcpyAsync(d, hb.data(), hb.size(), hipMemcpyHostToDevice, st));
  const unsigned char* db = (const unsigned char*)d;
  const int nt = lmats + lreal;
  hipLaunchKernelGGL(k_gf_poles, dim3((nt + kBlock - 1) / kBlock), dim3(kBlock), 0, st, (const GfFrac*)db, nfrac,
                     (const double*)(db + bf), (const double*)(db + bf + be), wm, lmats, wr, lreal, eps,
                     (double2*)gm, (double2*)gr);
  const hipError_t le = hipGetLastError();
  (void)hipFreeAsync(d, st);
  // the host staging vector dies on return: the copy must have completed
  HIPCK(hipStreamSynchronize(st));
  HIPCK(le);
  return ED_OK;
}

int ed_sector_lanc_tridiag_dev(ed_sector* s, int32_t vtype, const void* v0_dev, int32_t nitermax,
                               double threshold, double* alfa, double* beta, int32_t* nlanc) {
  if (!s || !alfa || !beta || !v0_dev || nitermax < 1) return fail(ED_ERR_ARG, "bad args");
  HIPCK(hipSetDevice(s->device));
  LancDriver d;
  CK(make_driver(s, vtype, false, &d));
  CK(lanc_prepare(s, d.vc, nitermax, false, 0));
  // v0_dev must be complete when this is called (the caller synchronises the
  // stream that produced it): no device-wide sync, which would fail while
  // another host thread captures a graph on its own sector stream
  CK(lanc_load_start(s, d.vc, v0_dev, true));
  CK(d.start(threshold));
  CK(d.iters(nitermax, true));
  std::vector<double> a(nitermax + 1), b(nitermax + 2);
  HIPCK(hipMemcpyAsync(a.data(), s->ws.alpha, nitermax * 8, hipMemcpyDeviceToHost, d.st));
  HIPCK(hipMemcpyAsync(b.data(), s->ws.beta, (nitermax + 1) * 8, hipMemcpyDeviceToHost, d.st));
  LancState hs;
  HIPCK(hipMemcpyAsync(&hs, s->ws.st, sizeof(hs), hipMemcpyDeviceToHost, d.st));
  HIPCK(hipStreamSynchronize(d.st));
  int n = hs.iter;
  for (int q = 0; q < nitermax; q++) {
    alfa[q] = q < n ? a[q] : 0.0;
    beta[q] = (q >= 1 && q <= n) ? b[q] : 0.0;
  }
  beta[0] = 0.0;
  if (nlanc) *nlanc = n;
  return ED_OK;
}

int ed_sector_lanc_eigh(ed_sector* s, int32_t vtype, const void* v0, int32_t nitermax,
                        double threshold, int32_t ncheck, double* egs, void* vect,
                        int32_t* nlanc) {
  if (!s || !egs || nitermax < 1) return fail(ED_ERR_ARG, "bad args");
  if (ncheck < 1) ncheck = 10;
  HIPCK(hipSetDevice(s->device));
  const int vc = vtype ? 1 : 0;
  const size_t vs = vc ? 16 : 8;
  // keep the Krylov basis when it fits in 1/4 of free memory (no second pass)
  size_t fr = 0, tot = 0;
  HIPCK(hipMemGetInfo(&fr, &tot));
  const bool keep = vect && ((double)nitermax * s->dim * vs < 0.25 * (double)fr);
  LancDriver d;
  CK(make_driver(s, vtype, keep, &d));
  CK(lanc_prepare(s, vc, nitermax, keep, keep ? nitermax : 0));
  CK(lanc_load_start(s, vc, v0, false));
  CK(d.start(threshold));
  // lanczos_plain_c convergence test, evaluated on the host between chunks
  std::vector<double> a(nitermax + 2, 0.0), b(nitermax + 2, 0.0), esave;
  int done_iters = 0, nl = 0;
  bool stop = false;
  const int chunk = d.pm >= 0 ? 64 : 32;
  while (!stop && done_iters < nitermax) {
    int n = std::min(chunk, nitermax - done_iters);
    const int expected = done_iters + n;
    CK(d.iters(n, done_iters == 0));
    HIPCK(hipMemcpyAsync(a.data(), s->ws.alpha, nitermax * 8, hipMemcpyDeviceToHost, d.st));
    HIPCK(hipMemcpyAsync(b.data(), s->ws.beta, (nitermax + 1) * 8, hipMemcpyDeviceToHost, d.st));
    LancState hs;
    HIPCK(hipMemcpyAsync(&hs, s->ws.st, sizeof(hs), hipMemcpyDeviceToHost, d.st));
    HIPCK(hipStreamSynchronize(d.st));
    int have = hs.iter;
    for (int it = done_iters + 1; it <= have && !stop; it++) {
      // iteration `it`: a = a[it-1], b = b[it]
      if (fabs(b[it]) < threshold) { stop = true; break; }
      nl = it;
      if (nl >= ncheck) {
        double e0 = lowest_ritz(a, b, nl);
        esave.push_back(e0);
        if (esave.size() >= 2 && fabs(esave.back() - esave[esave.size() - 2]) <= threshold) stop = true;
      }
    }
    if (hs.done) stop = true;
    if (have < expected && !hs.done) return fail(ED_ERR_STATE, "Lanczos iteration count mismatch");
    done_iters = have;
  }
  if (nl == 0) {
    LancState hs;
    CK(dcopy(s, &hs, s->ws.st, sizeof(hs), hipMemcpyDeviceToHost));
    char msg[256];
    snprintf(msg, sizeof msg,
             "Lanczos made no step: iter=%d done=%d beta0=%g b[1]=%g a[0]=%g path=%d pm=%d keep=%d",
             hs.iter, hs.done, hs.beta, b[1], a[0], d.path, d.pm, (int)keep);
    return fail(ED_ERR_STATE, msg);
  }
  // Ritz value and vector of the truncated tridiagonal (nl iterations)
  std::vector<double> dg(a.begin(), a.begin() + nl), e(nl, 0.0), z((size_t)nl * nl, 0.0);
  for (int q = 1; q < nl; q++) e[q] = b[q];
  for (int q = 0; q < nl; q++) z[q + (size_t)nl * q] = 1.0;
  if (nl > 0) tql2(nl, dg.data(), e.data(), z.data());
  *egs = nl > 0 ? dg[0] : 0.0;
  if (nlanc) *nlanc = nl;
  if (vect && nl > 0) {
    LancWS& w = s->ws;
    HIPCK(hipMemcpyAsync(w.z, z.data(), nl * 8, hipMemcpyHostToDevice, s->stream));  // Z(:,1)
    RedSlot slot{w.partials, w.counter + 2};
    if (keep) {
      if (vc)
        hipLaunchKernelGGL(k_ritz<true>, dim3(grid_once(s->dim)), dim3(kBlock), 0, s->stream,
                           (const double2*)w.basis, w.z, nl, s->dim, (double2*)w.Y, w.st, slot);
      else
        hipLaunchKernelGGL(k_ritz<false>, dim3(grid_once(s->dim)), dim3(kBlock), 0, s->stream,
                           (const double*)w.basis, w.z, nl, s->dim, (double*)w.Y, w.st, slot);
    } else {
      // second pass as lanczos_plain_c (:374-381): rerun the recurrence, y += Z(it,1) v_it
      // (multi-kernel recurrence: its P buffer holds v_it after each step)
      HIPCK(hipMemsetAsync(w.Y, 0, s->dim * vs, s->stream));
      CK(lanc_load_start(s, vc, v0, false));
      CK(vc ? lanc_start<true>(s, threshold, s->stream) : lanc_start<false>(s, threshold, s->stream));
      for (int it = 0; it < nl; it++) {
        CK(vc ? lanc_iter<true>(s, d.path, false, s->stream) : lanc_iter<false>(s, d.path, false, s->stream));
        if (vc)
          hipLaunchKernelGGL(k_axpy_p<true>, dim3(grid_for(s->dim)), dim3(kBlock), 0, s->stream,
                             (const double2*)w.P, w.z, it, s->dim, (double2*)w.Y);
        else
          hipLaunchKernelGGL(k_axpy_p<false>, dim3(grid_for(s->dim)), dim3(kBlock), 0, s->stream,
                             (const double*)w.P, w.z, it, s->dim, (double*)w.Y);
      }
      if (vc)
        hipLaunchKernelGGL(k_norm<true>, dim3(grid_once(s->dim)), dim3(kBlock), 0, s->stream,
                           (const double2*)w.Y, s->dim, w.st, slot);
      else
        hipLaunchKernelGGL(k_norm<false>, dim3(grid_once(s->dim)), dim3(kBlock), 0, s->stream,
                           (const double*)w.Y, s->dim, w.st, slot);
    }
    if (vc)
      hipLaunchKernelGGL(k_scale_tmp<true>, dim3(grid_for(s->dim)), dim3(kBlock), 0, s->stream,
                         (double2*)w.Y, s->dim, w.st);
    else
      hipLaunchKernelGGL(k_scale_tmp<false>, dim3(grid_for(s->dim)), dim3(kBlock), 0, s->stream,
                         (double*)w.Y, s->dim, w.st);
    HIPCK(hipGetLastError());
    HIPCK(hipMemcpyAsync(vect, w.Y, s->dim * vs, hipMemcpyDefault, s->stream));
    HIPCK(hipStreamSynchronize(s->stream));
  }
  return ED_OK;
}

int ed_sectors_eigh_batch(ed_sector* const* secs, int32_t n, int32_t nev, int32_t ncv, const int32_t* maxit,
                          double tol, const double* const* v0, double* evals, void* const* evecs, int32_t* nconv,
                          int32_t* nhv, int32_t* nbatched, int32_t flags, void* stream) {
  if (!secs || n < 0 || !evals || !maxit) return fail(ED_ERR_ARG, "bad args");
  for (int i = 0; i < n; i++)
    if (maxit[i] < 1) return fail(ED_ERR_ARG, "maxit < 1");
  if (n == 0) return ED_OK;
  if (ncv > kTrlanMaxCols) return fail(ED_ERR_ARG, "ncv > 64 not supported");
  for (int i = 0; i < n; i++) {
    if (!secs[i]) return fail(ED_ERR_ARG, "null sector");
    CK(whole_only(secs[i]));
    if (secs[i]->hc) return fail(ED_ERR_ARG, "batched eigh: real vectors only (complex H needs vtype=1)");
    if (secs[i]->device != secs[0]->device) return fail(ED_ERR_ARG, "batched eigh: sectors on different devices");
  }
  const int dev = secs[0]->device;
  HIPCK(hipSetDevice(dev));
  hipStream_t st = stream ? (hipStream_t)stream : secs[0]->stream;
  // up to kTbWgMaxDim rows: one workgroup per sector (ed_trlbatch.hpp), on a
  // second stream from a helper thread; larger: the lockstep multi-sector
  // solve (ed_trlmulti.hpp) here; the rest one by one afterwards
  std::vector<int> small, multi, fb, fb_small;
  for (int i = 0; i < n; i++) {
    if (secs[i]->dim <= kTbWgMaxDim && tb_eligible(secs[i], nev, ncv)) small.push_back(i);
    else if (tm_eligible(secs[i], nev, ncv)) multi.push_back(i);
    else fb.push_back(i);
  }
  int rc_small = ED_OK;
  std::string err_small;
  std::thread th;
  hipStream_t st2 = nullptr;
  if (!small.empty()) {
    if (multi.empty()) {
      rc_small = tb_run(secs, small, nev, ncv, maxit, tol, v0, evals, evecs, nconv, nhv, st, fb_small);
    } else {
      HIPCK(hipStreamCreateWithFlags(&st2, hipStreamNonBlocking));
      th = std::thread([&] {
        if (hipSetDevice(dev) != hipSuccess) rc_small = ED_ERR_HIP;
        else rc_small = tb_run(secs, small, nev, ncv, maxit, tol, v0, evals, evecs, nconv, nhv, st2, fb_small);
        if (rc_small != ED_OK) err_small = ed_err_slot();
      });
    }
  }
  int rc_multi = ED_OK;
  for (size_t c0 = 0; c0 < multi.size() && rc_multi == ED_OK; c0 += kTmMaxEntries) {
    const std::vector<int> part(multi.begin() + c0, multi.begin() + std::min(multi.size(), c0 + kTmMaxEntries));
    rc_multi = tm_run(secs, part, nev, ncv, maxit, tol, v0, evals, evecs, nconv, nhv, st, fb);
  }
  if (th.joinable()) th.join();
  if (st2) (void)hipStreamDestroy(st2);
  if (rc_multi != ED_OK) return rc_multi;
  if (rc_small != ED_OK) return fail(rc_small, err_small.empty() ? ed_err_slot() : err_small);
  fb.insert(fb.end(), fb_small.begin(), fb_small.end());
  if (nbatched) *nbatched = n - (int)fb.size();
  if (flags & ED_BATCH_NO_FALLBACK) {  // the caller solves them (nconv -1)
    for (int i : fb)
      if (nconv) nconv[i] = -1;
    return ED_OK;
  }
  for (int i : fb) {
    int32_t c = 0, h = 0;
    CK(trlan_run<false>(secs[i], nev, ncv, maxit[i], tol, v0 ? v0[i] : nullptr, evals + (size_t)i * nev,
                        evecs ? evecs[i] : nullptr, &c, &h));
    if (nconv) nconv[i] = c;
    if (nhv) nhv[i] += h;
  }
  return ED_OK;
}

int ed_sector_lanc_mode(ed_sector* s, int32_t vtype, int32_t path) {
  if (!s) {
    fail(ED_ERR_ARG, "null");
    return -2;
  }
  if (hipSetDevice(s->device) != hipSuccess) return -2;
  return persist_mode(s, vtype ? 1 : 0, resolve_path(s, path));
}

int ed_sector_eigh(ed_sector* s, int32_t vtype, int32_t nev, int32_t ncv, int32_t maxit,
                              double tol, const void* v0, double* evals, void* evecs, int32_t* nconv,
                              int32_t* nhv) {
  if (!s || !evals || maxit < 1) return fail(ED_ERR_ARG, "bad args");
  CK(whole_only(s));
  if (vtype == 0 && s->hc) return fail(ED_ERR_ARG, "complex H needs vtype=1");
  if (ncv > kTrlanMaxCols) return fail(ED_ERR_ARG, "ncv > 64 not supported");
  HIPCK(hipSetDevice(s->device));
  return vtype ? trlan_run<true>(s, nev, ncv, maxit, tol, v0, evals, evecs, nconv, nhv)
               : trlan_run<false>(s, nev, ncv, maxit, tol, v0, evals, evecs, nconv, nhv);
}

// ------------------------------------------------- reference-style globals
static std::mutex g_mu;
static ed_params g_params;
static bool g_have_params = false;
static int g_device = 0;
static ed_sector* g_cur = nullptr;

int ed_gpu_init(const ed_params* p) {
  if (!p) return fail(ED_ERR_ARG, "null params");
  EdModel M;
  int rc = model_from_params(p, &M);
  if (rc != ED_OK) return fail(rc, "invalid ed_params");
  std::lock_guard<std::mutex> lk(g_mu);
  g_params = *p;
  g_have_params = true;
  return ED_OK;
}

int ed_gpu_set_device(int32_t device) {
  int n = 0;
  HIPCK(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(ED_ERR_ARG, "bad device");
  g_device = device;
  return ED_OK;
}

int ed_gpu_build_sector(int32_t q1, int32_t q2, int32_t flags, int64_t* dim) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_have_params) return fail(ED_ERR_STATE, "ed_gpu_init not called");
  if (g_cur) {  // build_Hv_sector on a live sector: replace it
    sector_free(g_cur);
    g_cur = nullptr;
  }
  CK(ed_sector_create(&g_params, q1, q2, flags, g_device, nullptr, &g_cur));
  if (dim) *dim = g_cur->dim;
  return ED_OK;
}

int ed_gpu_vecdim(int32_t* vecdim) {
  if (!g_cur || !vecdim) return fail(ED_ERR_STATE, "no current sector");
  *vecdim = (int32_t)g_cur->nrows;  // MpiQ + MpiR (ED_HAMILTONIAN.f90:126-149); serial: Dim
  return ED_OK;
}

int ed_gpu_mpi_split(int64_t dim, int32_t rank, int32_t size, int64_t* row0, int64_t* nrows) {
  if (!row0 || !nrows || size < 1 || rank < 0 || rank >= size || dim < 0) return fail(ED_ERR_ARG, "mpi_split args");
  const int64_t q = dim / size;                          // MpiQ
  const int64_t r = rank == size - 1 ? dim % size : 0;   // MpiR (last rank)
  *row0 = (int64_t)rank * q;                             // MpiIshift
  *nrows = q + r;                                        // MpiIend - MpiIstart + 1
  return ED_OK;
}
int ed_gpu_build_sector_rows(int32_t q1, int32_t q2, int32_t flags, int64_t row0, int64_t nrows, int64_t* dim) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (!g_have_params) return fail(ED_ERR_STATE, "ed_gpu_init not called");
  if (g_cur) {
    sector_free(g_cur);
    g_cur = nullptr;
  }
  CK(ed_sector_create_rows(&g_params, q1, q2, flags, row0, nrows, g_device, nullptr, &g_cur));
  if (dim) *dim = g_cur->dim;
  return ED_OK;
}
int ed_gpu_hxv_mpi(const int32_t* nloc, const double* vin, double* hv) {
  if (!g_cur) return fail(ED_ERR_STATE, "ed_gpu_hxv_mpi ERROR: Hsector NOT set");
  if (!nloc) return fail(ED_ERR_ARG, "null");
  ed_sector* s = g_cur;
  if ((int64_t)*nloc != s->nrows) return fail(ED_ERR_ARG, "ed_gpu_hxv_mpi ERROR: Nloc != local rows of the sector");
  if (s->nrows == 0) return ED_OK;
  if (!vin || !hv) return fail(ED_ERR_ARG, "null");
  HIPCK(hipSetDevice(s->device));
  if (!s->d_x) {
    CK(dalloc(s, &s->d_x, s->dim * 16));
    CK(dalloc(s, &s->d_y, s->nrows * 16));
  }
  HIPCK(hipMemcpyAsync(s->d_x, vin, s->dim * 16, hipMemcpyHostToDevice, s->stream));
  CK(ed_sector_hxv_dev(s, 1, s->d_x, s->d_y, s->stream));
  HIPCK(hipMemcpyAsync(hv, s->d_y, s->nrows * 16, hipMemcpyDeviceToHost, s->stream));
  HIPCK(hipStreamSynchronize(s->stream));
  return ED_OK;
}
int ed_gpu_hxv(const int32_t* nloc, const double* v, double* hv) {
  if (!g_cur) return fail(ED_ERR_STATE, "ed_gpu_hxv ERROR: Hsector NOT set");
  if (!nloc) return fail(ED_ERR_ARG, "null nloc");
  return ed_sector_hxv(g_cur, *nloc, v, hv);
}

int ed_gpu_dump_csr(int64_t* rowptr, int32_t* cols, double* vals) {
  if (!g_cur) return fail(ED_ERR_STATE, "no current sector");
  return ed_sector_dump_csr(g_cur, rowptr, cols, vals);
}

int ed_gpu_lanc_eigh(int32_t nitermax, double threshold, int32_t ncheck, double* egs, double* vect,
                     int32_t* nlanc) {
  if (!g_cur) return fail(ED_ERR_STATE, "no current sector");
  return ed_sector_lanc_eigh(g_cur, 1, nullptr, nitermax, threshold, ncheck, egs, vect, nlanc);
}

int ed_gpu_eigh(int32_t neigen, int32_t nblock, int32_t nitermax, double tol, const double* v0,
                double* evals, double* evecs, int32_t* nconv) {
  if (!g_cur) return fail(ED_ERR_STATE, "no current sector");
  const int64_t dim = g_cur->dim;
  const int ncv = (int)std::min<int64_t>(std::min(std::max(nblock, neigen + 1), 64), dim);
  return ed_sector_eigh(g_cur, 1, neigen, ncv, nitermax, tol, v0, evals, evecs, nconv, nullptr);
}

int ed_gpu_lanc_tridiag(const double* v0, int32_t nitermax, double threshold, double* alfa,
                        double* beta, int32_t* nlanc) {
  if (!g_cur) return fail(ED_ERR_STATE, "no current sector");
  return ed_sector_lanc_tridiag(g_cur, 1, v0, nitermax, threshold, alfa, beta, nlanc);
}

int ed_gpu_delete_sector(void) {
  std::lock_guard<std::mutex> lk(g_mu);
  // delete_Hv_sector: safe after a direct build (the reference stops in
  // sp_delete_matrix there, ED_HAMILTONIAN.f90:111-119 / ED_SPARSE_MATRIX.f90:180)
  if (g_cur) sector_free(g_cur);
  g_cur = nullptr;
  return ED_OK;
}

int ed_gpu_finalize(void) {
  ed_gpu_delete_sector();
  std::lock_guard<std::mutex> lk(g_mu);
  g_have_params = false;
  return ED_OK;
}

int ed_gpu_current_sector(ed_sector** out) {
  if (!out) return fail(ED_ERR_ARG, "null");
  *out = g_cur;
  return g_cur ? ED_OK : fail(ED_ERR_STATE, "no current sector");
}

}  // extern "C"
