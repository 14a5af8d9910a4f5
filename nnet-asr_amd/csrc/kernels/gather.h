// gather.h -- the next bunch's gather as workgroups of another launch (the step's last update, the data-parallel
// step's last gradient GEMM, the softmax launch): CuCache::GetBunch's row gather by the shuffled permutation
// (cuCache.cc:155-200) for a class-id target cache.
#pragma once

#include "kcommon.h"

namespace tnetk {

// The next bunch's gather (tnet_gather_bunch: bunch row r = cache row idx[r], its class id alongside) as
// workgroups of the step's last update launch.  Wave w of ngb*4 takes rows w, w + ngb*4, ...; R rows at a
// time with every 16-B load of those rows issued before the first store (the rows' idx loads before
// that), so a wave pays two memory round trips per R rows.  c4 = cols rounded up to 4 (16-B pieces; the
// caller checked that both strides hold them).
struct BunchGatherP {
  float* y;
  const float* x;
  int* lab_out;
  const int* lab_in;
  const int* idx;
  int rows, c4;
  long ys, xs;
};
__device__ __forceinline__ void bunch_gather_block(const BunchGatherP& g, const int gb, const int ngb) {
  constexpr int R = 4, CM = 2;  // rows and 256-column pieces per lane in flight
  const int lane = threadIdx.x & 63, nw = blockDim.x >> 6;
  const int w0 = gb * nw + (threadIdx.x >> 6), step = ngb * nw;
  for (int r0 = w0; r0 < g.rows; r0 += R * step) {
    int ir[R];
#pragma unroll
    for (int k = 0; k < R; ++k) ir[k] = r0 + k * step < g.rows ? g.idx[r0 + k * step] : -1;
#pragma unroll
    for (int k = 0; k < R; ++k)
      if (ir[k] >= 0 && lane == 0) g.lab_out[r0 + k * step] = g.lab_in[ir[k]];
    for (int cb = lane * 4; cb < g.c4; cb += 256 * CM) {
      f32x4 v[R][CM];
#pragma unroll
      for (int k = 0; k < R; ++k)
#pragma unroll
        for (int j = 0; j < CM; ++j)
          if (ir[k] >= 0 && cb + 256 * j < g.c4) v[k][j] = *reinterpret_cast<const f32x4*>(g.x + ir[k] * g.xs + cb + 256 * j);
#pragma unroll
      for (int k = 0; k < R; ++k) {
        if (ir[k] < 0) continue;
        // the bunch row written through (st_wt): the next step's first GEMM reads it on every XCD
        const __amdgpu_buffer_rsrc_t ry = tile_rsrc(g.y + (long)(r0 + k * step) * g.ys);
#pragma unroll
        for (int j = 0; j < CM; ++j)
          if (cb + 256 * j < g.c4) st_wt(ry, cb + 256 * j, v[k][j]);
      }
    }
  }
}

}  // namespace tnetk
