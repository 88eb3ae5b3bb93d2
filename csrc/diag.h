// The one diagnostic switchboard of the native code: DISTRIFLOW_DIAG="name=value,name=value".
//
// Measurement aids only (A/B of kernel variants that were measured neutral or slower, tile-size
// sweeps): production never sets DISTRIFLOW_DIAG, and every switch defaults to the shipped path.  Kept
// in one place so that the alternative code paths are discoverable and documented (docs/RESULTS.md);
// the Python side reads the same variable through distriflow_amd/diagnostics.py.
//   igemm_fast=0    igemm64 without the FAST gather           igemm_splitk=0  igemm64 without split-K
//   bn_rpt=N        BatchNorm statistics rows per thread      wgrad_wg=N      wgrad_tr workgroup target
//   bn_max_g=N      BatchNorm statistics workgroup cap (16..1008, default 255)
//   wgrad128=N      wgrad_tr 128x128 tile rows per step       cp_wpc=N        convpool workgroups per CU cap
//   cp_minimgs=N    convpool images per workgroup floor
//   wgrad_halo=0    3x3 weight gradients on wgrad_tr instead of the halo kernel
//   halo_groups=1   halo weight gradient with 4-wave workgroups (default: two groups sharing a slab)
//   halo_wg=N       halo weight-gradient workgroup target    conv_halo=0     3x3 fwd/dgrad on igemm64
//   conv_halo_c64=0 no weights-resident 64->64 kernel        conv_halo_splitk=0 / conv_halo_ks=N
//   conv_halo_fold=0 two-split halo convs combined by a separate launch (default: the last arriver)
//                                                            halo fwd/dgrad channel-block split (max N)
#pragma once
#include <cstdlib>
#include <cstring>

namespace dfa {

inline int diag_int(const char* name, int dflt) {
  const char* s = getenv("DISTRIFLOW_DIAG");
  if (!s || !*s) return dflt;
  const size_t n = strlen(name);
  while (*s) {
    while (*s == ',' || *s == ' ') ++s;
    if (strncmp(s, name, n) == 0 && s[n] == '=') return atoi(s + n + 1);
    while (*s && *s != ',') ++s;
  }
  return dflt;
}

}  // namespace dfa
