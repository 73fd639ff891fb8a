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
// (combinatorial number system; for Jz_basis sectors among the patterns of
// the same (popcount, Lz)) and off[idw] = number of sector states in the
// blocks before idw.  Two 2^Ns tables (<= 256 KB each at Ns=16) replace the
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
  int jz = 0;                     // Jz_basis sector (n, twoJz)
  int64_t dim = 0;
  // Patterns of one spin are grouped in classes: the popcount, or for Jz
  // sectors (popcount, 2*Lz) -- an idw block of the sector takes exactly the
  // iup of one class, in ascending order.
  std::vector<int32_t> cls;       // [nst] class of each pattern
  std::vector<uint32_t> rank;     // [nst] position of x among the patterns of its class
  std::vector<int32_t> off;       // [nst], -1: idw has no state in the sector
  std::vector<int32_t> need_cls;  // [nst], class of iup required by idw, -1 if none
  std::vector<uint32_t> by_cls;   // [nst] patterns sorted by (class, value)
  std::vector<int32_t> cls_start; // [ncls+1]
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

// lz2: 2*Lzdiag per level for a Jz_basis sector (q1 = n, q2 = twoJz), else null.
// Jz: twoJz = (nup - ndw) + lz2(iup) + lz2(idw) (build_sector ED_SETUP.f90:940-965).
inline int build_tables(int ns, int mode, int q1, int q2, SectorTables* T, const int32_t* lz2 = nullptr) {
  if (ns < 1 || ns > ED_MAX_NS) return ED_ERR_ARG;
  T->ns = ns;
  T->nst = 1u << ns;
  T->mode = mode; T->q1 = q1; T->q2 = q2;
  T->jz = lz2 ? 1 : 0;
  const uint32_t nst = T->nst;
  const int LO = 2 * ns, LW = 4 * ns + 1;  // 2*Lz in [-2Ns, 2Ns]
  const int ncls = lz2 ? (ns + 1) * LW : ns + 1;
  std::vector<int32_t> lzp(lz2 ? nst : 0, 0);
  T->cls.assign(nst, 0);
  for (uint32_t x = 0; x < nst; x++) {
    const int pc = __builtin_popcount(x);
    if (lz2) {
      int l = 0;
      for (int b = 0; b < ns; b++)
        if ((x >> b) & 1u) l += lz2[b];
      lzp[x] = l;
      T->cls[x] = pc * LW + l + LO;
    } else {
      T->cls[x] = pc;
    }
  }
  T->rank.assign(nst, 0);
  T->off.assign(nst, -1);
  T->need_cls.assign(nst, -1);
  T->by_cls.assign(nst, 0);
  T->cls_start.assign(ncls + 1, 0);
  std::vector<int32_t> cnt(ncls, 0);
  for (uint32_t x = 0; x < nst; x++) T->rank[x] = (uint32_t)cnt[T->cls[x]]++;  // ascending x in a class
  for (int c = 0; c < ncls; c++) T->cls_start[c + 1] = T->cls_start[c] + cnt[c];
  for (uint32_t x = 0; x < nst; x++) T->by_cls[T->cls_start[T->cls[x]] + T->rank[x]] = x;
  int64_t dim = 0;
  T->blk_off.clear();
  T->blk_idw.clear();
  for (uint32_t idw = 0; idw < nst; idw++) {
    const int pd = __builtin_popcount(idw);
    int nup = required_nup(mode, q1, q2, pd, ns);
    if (nup < 0) continue;
    int c = nup;
    if (lz2) {
      const int lu = q2 - (nup - pd) - lzp[idw];
      if (lu < -LO || lu > LO) continue;
      c = nup * LW + lu + LO;
    }
    const int64_t b = cnt[c];
    if (b == 0) continue;
    if (dim + b > INT32_MAX) return ED_ERR_UNSUPPORTED;  // int32 columns
    T->off[idw] = (int32_t)dim;
    T->need_cls[idw] = c;
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
  const uint32_t idw = k >> T.ns, iup = k & (T.nst - 1);
  const int32_t o = T.off[idw];
  if (o < 0 || T.cls[iup] != T.need_cls[idw]) return -1;
  return (int64_t)o + T.rank[iup];
}

}  // namespace edg
