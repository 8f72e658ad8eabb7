// ocx_exact_src.h — where the general exact solvers (ocx_exact_wide.hip, d <= 64;
// ocx_exact_big.hip, 64 < d <= 256) read a problem's rows and labels: row-major z [B][T][d] /
// y [B][T], or the tiled layout of include/ocx.h (P, C, S, G of it).
#pragma once

#include <cstdint>

#include <hip/hip_runtime.h>

// element (i, j) of sequence b's rows: row-major z [B][T][d] or the tiled layout
struct WideSrc {
    const double* z;
    const double* y;
    int64_t T, G;
    int d, P, C, S, tiled;
    __device__ __forceinline__ double zat(int64_t b, int64_t i, int j) const {
        if (!tiled) return z[(b * T + i) * d + j];
        const int64_t g = b / S;
        const int s = (int)(b - g * S);
        const int jl = j / C, jj = j - jl * C;
        return z[((int64_t)(jj >> 1) * G + g) * T * 128 + i * 128 + 2 * (s * P + jl) + (jj & 1)];
    }
    __device__ __forceinline__ double yat(int64_t b, int64_t i) const {
        if (!tiled) return y[b * T + i];
        const int64_t g = b / S;
        return y[(g * T + i) * S + (b - g * S)];
    }
};
