// One documented switch for A/B measurements of the kernel geometry and the
// issue rules (development aid; production runs never set it):
//
//   SVDJ_DEBUG="key=value[,key=value...]"
//     merge=0|1            one-GPU merged issue of the two chains forced off/on
//                          (world 1 only, both engines: svdj_dist_issue_rules,
//                          parallel/distributed.py choose_merged)
//     gram_chunks=N        row chunks of the single-step Gram (make_geometry)
//     quad_gram_chunks=N   row chunks of the quad Gram (quad_geometry)
//     stream_order=B       row-chunk dispatch order: bit 0 cross Gram chunks
//                          last-first, bit 1 the apply's V chunks before A's
//     cheap_log2=K         quad apply: first-order-only k halves where
//                          |T - I| <= 2^-K (default 7)
//     qb1_threads=N        phase-1 quad Q build workgroup size (1024 or 512)
//     upd_threads=N        quad_update_kernel workgroup size (256 or 512)
//     cross_reduce_chunks=N  single cross steps (fp32 W = 64): pre-sum the Gram's
//                          row chunks when there are at least N (default 9)
//     gram2=0|1            quad Gram on 2 bf16 parts forced off / on (default:
//                          while the previous sweep rotated every pair; both
//                          engines: parallel/distributed.py, svdj_dist_solve)
//     apply_grid=N         quad apply persistent grid (default 256 = one
//                          workgroup per CU)
//     quad_pad=0           no extra zero columns for quad steps (both engines'
//                          geometry: svdj_dist_geometry, distributed.py)
//
// svdj_debug_knob returns the value of `key`, or `dflt` when SVDJ_DEBUG is
// unset or does not name it.  Host code only; callers cache the result.
// The Python twin is config.debug_knob.
#pragma once
#include <stdlib.h>
#include <string.h>

static inline int svdj_debug_knob(const char* key, int dflt) {
  const char* e = getenv("SVDJ_DEBUG");
  if (!e) return dflt;
  const size_t kl = strlen(key);
  for (const char* p = e; *p;) {
    const char* end = strchr(p, ',');
    const size_t len = end ? (size_t)(end - p) : strlen(p);
    if (len > kl && strncmp(p, key, kl) == 0 && p[kl] == '=') return atoi(p + kl + 1);
    if (!end) break;
    p = end + 1;
  }
  return dflt;
}
