// ed_tables.hpp — Fock-basis index tables of one symmetry sector (host side).
//
// The reference enumerates a sector by scanning all 2^Ns x 2^Ns (iup, idw)
// pairs with idw outer, iup inner, keeping those with the right quantum
// numbers, and stores the kept states in the ascending array H%map
// (build_sector, ED_SETUP.f90:886-984).  It then finds a state's row by
// recursive binary search over H%map (binary_search, ED_SETUP.f90:1307-1324).
//
// Because idw is the outer loop, the states sharing one idw form a contiguous
// block, and inside a block the iup are in ascending order among patterns of
// one fixed popcount.  So the row of state k = iup + idw*2^Ns is
//     index(k) = off[idw] + rank[iup]            (0-based)
// with rank[x] = position of x among the Ns-bit patterns of popcount(x)
// (combinatorial number system) and off[idw] = number of sector states in
// the blocks before idw.  Two 2^Ns tables (<= 256 KB each at Ns=16) replace the
// O(log dim) search, and map[i] itself is produced on the device from
// (off, rank) — see k_build_map in ed_kernels.hpp.
#pragma once
#include <stdint.h>

#include <vector>

#include "ed_model.hpp"

namespace edg {

inline int64_t binom64(int n, int k) {
  if (k < 0 || k > n) return 0;
  int64_t r = 1;
  for (int i = 1; i <= k; i++) r = r * (n + 1 - i) / i;
  return r;
}

struct SectorTables {
  int ns = 0;
  uint32_t nst = 0;               // 2^Ns
  int mode = 0, q1 = 0, q2 = 0;
  int64_t dim = 0;
  std::vector<uint32_t> rank;     // [nst]
  std::vector<int32_t> off;       // [nst], -1: idw has no state in the sector
  std::vector<int32_t> need_nup;  // [nst], popcount(iup) required by idw, -1 if none
  std::vector<uint32_t> by_pc;    // [nst] patterns sorted by (popcount, value)
  std::vector<int32_t> pc_start;  // [ns+2]
  std::vector<int64_t> blk_off;   // [nblk+1] start row of each non-empty idw block
  std::vector<uint32_t> blk_idw;  // [nblk]
  // normal mode factorisation (DimUp x DimDw), else 0
  int64_t dimup = 0, dimdw = 0;
};

// Required popcount of iup for a given popcount of idw (-1 if none).
inline int required_nup(int mode, int q1, int q2, int ndw, int ns) {
  int nup;
  if (mode == ED_MODE_NORMAL) {
    if (ndw != q2) return -1;
    nup = q1;
  } else if (mode == ED_MODE_SUPERC) {
    nup = q1 + ndw;  // sz = nup - ndw
  } else {
    nup = q1 - ndw;  // n = nup + ndw
  }
  return (nup < 0 || nup > ns) ? -1 : nup;
}

inline int build_tables(int ns, int mode, int q1, int q2, SectorTables* T) {
  if (ns < 1 || ns > ED_MAX_NS) return ED_ERR_ARG;
  T->ns = ns;
  T->nst = 1u << ns;
  T->mode = mode; T->q1 = q1; T->q2 = q2;
  const uint32_t nst = T->nst;
  T->rank.assign(nst, 0);
  T->off.assign(nst, -1);
  T->need_nup.assign(nst, -1);
  T->by_pc.assign(nst, 0);
  T->pc_start.assign(ns + 2, 0);
  std::vector<int32_t> cnt(ns + 1, 0);
  for (uint32_t x = 0; x < nst; x++) {
    int pc = __builtin_popcount(x);
    T->rank[x] = (uint32_t)cnt[pc]++;  // ascending x within one popcount class
  }
  for (int pc = 0; pc <= ns; pc++) T->pc_start[pc + 1] = T->pc_start[pc] + cnt[pc];
  for (uint32_t x = 0; x < nst; x++) {
    int pc = __builtin_popcount(x);
    T->by_pc[T->pc_start[pc] + T->rank[x]] = x;
  }
  int64_t dim = 0;
  T->blk_off.clear();
  T->blk_idw.clear();
  for (uint32_t idw = 0; idw < nst; idw++) {
    int nup = required_nup(mode, q1, q2, __builtin_popcount(idw), ns);
    if (nup < 0) continue;
    int64_t b = binom64(ns, nup);
    if (b == 0) continue;
    if (dim + b > INT32_MAX) return ED_ERR_UNSUPPORTED;  // int32 columns
    T->off[idw] = (int32_t)dim;
    T->need_nup[idw] = nup;
    T->blk_off.push_back(dim);
    T->blk_idw.push_back(idw);
    dim += b;
  }
  T->blk_off.push_back(dim);
  T->dim = dim;
  if (mode == ED_MODE_NORMAL) {
    T->dimup = binom64(ns, q1);
    T->dimdw = binom64(ns, q2);
  }
  return ED_OK;
}

// Row index of a Fock state (0-based), -1 if outside the sector.
inline int64_t table_index(const SectorTables& T, uint32_t k) {
  int32_t o = T.off[k >> T.ns];
  if (o < 0) return -1;
  uint32_t iup = k & (T.nst - 1);
  if (__builtin_popcount(iup) != T.need_nup[k >> T.ns]) return -1;
  return (int64_t)o + T.rank[iup];
}

}  // namespace edg
