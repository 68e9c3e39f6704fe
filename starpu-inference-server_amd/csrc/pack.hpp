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
}

}  // namespace spi
