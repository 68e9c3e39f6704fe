// Host-side weight packing shared by model replicas and the op-level API.
#pragma once
#include <cstddef>
#include <cstring>

#include "spi_kernels.hpp"

namespace spi {

inline int round_up_to(int v, int m) { return (v + m - 1) / m * m; }

inline size_t packed_bytes(Prec prec, int Npad, int Kpad) {
  return (size_t)Npad * Kpad * (prec == Prec::F16 ? 2 : 4);
}

// Whether pack_matrix_into writes the weight-resident conv's LDS image into the padding
// rows (below): exactly the fp16 64 x 576 matrices.  A GemmDesc whose W came from such a
// pack says so with GemmDesc::w_image, and only then may conv_wres read those rows.
inline bool packed_has_wres_image(Prec prec, int N, int K, int Npad, int Kpad) {
  return prec == Prec::F16 && N == 64 && K == 576 && Npad == 128 && Kpad == 576;
}

// [N][K] -> [Npad][Kpad] in the compute layout; get(n, k) returns element (n, k).
// F16X3 rows are Kpad/32 blocks of [32 hi fp16 | 32 lo fp16] (lo = v - hi).
template <typename F>
void pack_matrix_into(char* dst, int N, int K, int Npad, int Kpad, Prec prec, F get) {
  std::memset(dst, 0, packed_bytes(prec, Npad, Kpad));
  for (int n = 0; n < N; ++n)
    for (int k = 0; k < K; ++k) {
      const float v = get(n, k);
      if (prec == Prec::F32) {
        reinterpret_cast<float*>(dst)[(size_t)n * Kpad + k] = v;
      } else if (prec == Prec::F16) {
        reinterpret_cast<_Float16*>(dst)[(size_t)n * Kpad + k] = static_cast<_Float16>(v);
      } else {
        const _Float16 hi = static_cast<_Float16>(v);
        _Float16* row = reinterpret_cast<_Float16*>(dst) + (size_t)n * 2 * Kpad + (size_t)(k / 32) * 64 + (k % 32);
        row[0] = hi;
        row[32] = static_cast<_Float16>(v - static_cast<float>(hi));
      }
    }
  // A 64 x 576 fp16 matrix (a 3x3 conv over 64 channels, k = tap * 64 + c) leaves its 64
  // padding rows unused by every GEMM tile that can run it (N = 64: one 64-column tile):
  // they hold the weight-resident conv's LDS image instead (conv_wres.hip) -- per tap t,
  // row n, 16-byte slot s: chunk s ^ (n & 7) of W[n][t * 64 ...] -- so that kernel fills
  // its LDS with 72 contiguous 1-KiB pieces.
  if (packed_has_wres_image(prec, N, K, Npad, Kpad)) {
    const _Float16* w = reinterpret_cast<const _Float16*>(dst);
    _Float16* img = reinterpret_cast<_Float16*>(dst) + (size_t)64 * Kpad;
    for (int t = 0; t < 9; ++t)
      for (int n = 0; n < 64; ++n)
        for (int sl = 0; sl < 8; ++sl) {
          const int c = sl ^ (n & 7);
          for (int e = 0; e < 8; ++e) img[((size_t)t * 64 + n) * 64 + sl * 8 + e] = w[(size_t)n * Kpad + t * 64 + c * 8 + e];
        }
  }
}

}  // namespace spi
