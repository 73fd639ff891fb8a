// ed_host.hpp — host-side pieces shared by the library's translation units:
// error reporting (ed_gpu_last_error's thread-local message), the HIPCK / CK
// early-return macros, the register budgets of the persistent kernels, and
// the persistent-launch dispatcher (ed_persist_launch.hip: the k_lanc_persist
// instantiations live in their own translation unit so the two halves of the
// library compile in parallel).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>

#include "../../include/ed_gpu.h"

std::string& ed_err_slot();
static inline int fail(int code, const std::string& msg) {
  ed_err_slot() = msg;
  return code;
}
#define HIPCK(x)                                                                       \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess)                                                              \
      return fail(ED_ERR_HIP, std::string(#x) + " -> " + hipGetErrorString(e_));       \
  } while (0)
#define CK(x)                  \
  do {                         \
    int r_ = (x);              \
    if (r_ != ED_OK) return r_; \
  } while (0)

namespace edg {

// Kronecker register layout (MODE 4): rows per thread that fit the register
// budget with E hop slots (real vectors)
constexpr bool pkr_fits(int E, int RPT) { return RPT * (3 * E + 8) + 3 * E <= 216; }
// complex vectors, 512-thread layout (-Rpass-analysis: spill-free forms)
constexpr bool pkr_fits_c512(int E, int RPT) { return E == 4 ? RPT <= 10 : RPT <= 6; }
// register-resident ELL words per thread (MODE 2/3) without spills
constexpr int preg_cap(bool hc, bool vc) { return vc ? (hc ? 80 : 84) : 112; }
// Rows per thread of the 1024-thread modes (0, 1): the launch's template value
static inline int persist_rpt01(int64_t dim) {
  const int64_t rpt = (dim + 1024 - 1) / 1024;
  return rpt <= 6 ? (int)rpt : rpt <= 8 ? 8 : rpt <= 10 ? 10 : rpt <= 12 ? 12 : 16;
}

// The sector fields that pick a k_lanc_persist instantiation
struct PersistGeom {
  int64_t dim = 0;
  int preg_E = 0, preg_rpt = 0, kreg_W = 0, kreg_rpt = 0, pkr_E = 0, pkr_rpt = 0;
};

// Launch k_lanc_persist for (hc, vc, mode) on the geometry's template values;
// run points to a PersistRun<hc>.
int persist_launch(bool hc, bool vc, int mode, const PersistGeom& g, const void* run, int64_t lds,
                   hipStream_t st, int nb);

}  // namespace edg
