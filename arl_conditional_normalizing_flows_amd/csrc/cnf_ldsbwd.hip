// cnf_ldsbwd.hip — fused training backward of a k_net_lds layer's s,t networks
// (conv_cINN_make_model.py:1076-1213 under the tf.GradientTape of train_step, :1850-1870).
//
// One workgroup per (image, net) walks the network in reverse with every gradient resident in LDS:
// conv_out, LN_out, then per residual block (last first) conv_b, LN3, the grouped dilated branches,
// LN2, conv_a, LN1 (the residual adds the identity path), and conv_in. The forward activations it
// needs are the raw tensors and LN statistics the training forward's k_net_lds saved (LdsSave), so
// nothing is recomputed; LN is LayerNormalization over H*W*C per image of LeakyReLU(x)
// (conv_cINN_base_functions.py:330-362). Data gradients are implicit GEMMs on
// v_mfma_f32_16x16x4_f32 over the transposed weights (3x3 taps mirrored through a k-table); weight
// gradients contract over the image's pixels on MFMA. Every parameter gradient of the image goes to
// its (net, image) row of the partial buffer in the net's canonical parameter order (convs through
// the dense backward map), and k_grad_rows sums the rows over the batch in a fixed order: the result is
// bitwise reproducible. This replaces the ~230 launches per layer of the multi-kernel backward
// (cnf_train.cpp) — one launch per layer plus the row sum.
//
// LDS (floats): GY [HW][sy] dL/dy (the residual stream's gradient) | GT [HW][st] dL/dt2, dL/dt1,
// dL/d(so) | AC [HW][sa] staged activations / the next gradient | W [kp][np] transposed weights |
// KT k-table ints | RED fp64 reduction scratch.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cnf_device.h"
#include "cnf_kernels.h"

namespace cnf {

namespace {

constexpr int BWN = 8;          // waves per workgroup
constexpr int BWT = BWN * 64;   // threads

__device__ __forceinline__ float lrelu_b(float x) { return lrelu(x); }   // (cnf_device.h)
__device__ __forceinline__ float lrelu_d(float x) { return x > 0.f ? 1.f : LRELU_ALPHA; }

// k-table entry of a flat reduction index k = tap * cpt + c: (dr + 64) | (dc + 64) << 7 | c << 14,
// dr / dc the pixel offset of the tap (sgn = +1: x[p + d*off], the forward taps; sgn = -1: the
// transposed conv's mirrored taps); -1 beyond K
__device__ __forceinline__ void build_kt(int* kt, int K, int Kp, int cpt, int taps, int d, int sgn) {
    for (int k = threadIdx.x; k < Kp; k += BWT) {
        int t = -1;
        if (k < K) {
            const int tap = k / cpt, c = k - tap * cpt;
            const int dr = taps == 9 ? sgn * d * (tap / 3 - 1) : 0, dc = taps == 9 ? sgn * d * (tap % 3 - 1) : 0;
            t = (dr + 64) | ((dc + 64) << 7) | (c << 14);
        }
        kt[k] = t;
    }
}

// A(p, k) of a k-table entry t for pixel (pr, pc): a[(p + shift) * sa + a_off + c], 0 outside the image
constexpr int KT_ONE = -2;   // k-table entry of the bias row of a weight gradient: A = 1

__device__ __forceinline__ float kt_load(const float* a, int sa, int a_off, int t, int pr, int pc, int H, int W) {
    if (t < 0) return t == KT_ONE ? 1.f : 0.f;
    const int y = pr + (t & 127) - 64, x = pc + ((t >> 7) & 127) - 64;
    if ((unsigned)y >= (unsigned)H || (unsigned)x >= (unsigned)W) return 0.f;
    return a[(y * W + x) * sa + a_off + (t >> 14)];
}

// LDS address of A(p, k) for k-table entry t and pixel (pr, pc) (pv: the pixel exists): the element,
// else the zero slot Z, or the one slot Z + 4 for the bias row (t == KT_ONE) — every operand is a load,
// so a group's loads issue together with no branch between them
__device__ __forceinline__ const float* kt_ptr(const float* a, int sa, int a_off, int t, int pr, int pc, bool pv,
                                               int H, int W, const float* Z) {
    const int y = pr + (t & 127) - 64, x = pc + ((t >> 7) & 127) - 64;
    const bool in = t >= 0 && pv && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
    return in ? a + (y * W + x) * sa + a_off + (t >> 14) : (t == KT_ONE && pv ? Z + 4 : Z);
}

// out[p][o_off + n] (= or +=) sum over taps t and channels c < cpt of A[p + shift(t)][a_off + c] *
// Wl[t * cpt4 + c][n] (cpt4 = cpt rounded up to 4; Wl's rows cpt..cpt4-1 of every tap are zero, and
// the A values they meet are finite: LDS is zeroed at kernel start), shift(t) = sgn * d * (t / 3 - 1,
// t % 3 - 1) for 3x3 convs. Units of SUB 16-pixel subtiles x NR 16-column blocks, dealt round-robin over
// the waves; per tap the lane's shifted row pointer (or the zero row Z) is computed once, so a k-step
// is one A load, NR B loads and NR x SUB MFMAs (no per-step table or address arithmetic).
// acc[s][m][r] = out[p0(s) + 4kq + r][n0 + 16m + i16].
template <int NR, int SUB>
__device__ void gemm_tap(const float* a, int sa, int a_off, int taps, int cpt4, int d, int sgn, const float* wl, int np,
                         float* out, int so, int o_off, int N, int H, int W, bool accum, const float* Z) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i16 = lane & 15, kq = lane >> 4;
    const int HW = H * W, nsub = (HW + 15) >> 4, ngrp = (np / 16 + NR - 1) / NR, nsg = (nsub + SUB - 1) / SUB;
    const float invW = 1.f / (float)W;
    for (int unit = wave; unit < nsg * ngrp; unit += BWN) {
        const int sg = unit % nsg, n0 = (unit / nsg) * 16 * NR;
        const int nb = min(NR, (np - n0) >> 4);   // column blocks of this unit (uniform)
        int pr[SUB], pc[SUB];
        bool pv[SUB];
#pragma unroll
        for (int s = 0; s < SUB; s++) {
            const int p = (sg * SUB + s) * 16 + i16;
            pv[s] = p < HW;
            pr[s] = (int)(((float)p + 0.5f) * invW);
            pc[s] = p - pr[s] * W;
        }
        f4 acc[SUB][NR];
#pragma unroll
        for (int s = 0; s < SUB; s++)
#pragma unroll
            for (int m = 0; m < NR; m++) acc[s][m] = f4{0.f, 0.f, 0.f, 0.f};
        for (int t = 0; t < taps; t++) {
            const int dr = taps == 9 ? sgn * d * (t / 3 - 1) : 0, dc = taps == 9 ? sgn * d * (t % 3 - 1) : 0;
            const float* ab[SUB];
#pragma unroll
            for (int s = 0; s < SUB; s++) {
                const int y = pr[s] + dr, x = pc[s] + dc;
                const bool in = pv[s] && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
                ab[s] = (in ? a + (y * W + x) * sa + a_off : Z) + kq;
            }
            const float* wt = wl + ((size_t)t * cpt4 + kq) * np + n0 + i16;
            int c = 0;
            for (; c + 16 <= cpt4; c += 16) {
                float av[4][SUB], bv[4][NR];
#pragma unroll
                for (int j = 0; j < 4; j++) {
#pragma unroll
                    for (int s = 0; s < SUB; s++) av[j][s] = ab[s][c + 4 * j];
#pragma unroll
                    for (int m = 0; m < NR; m++) bv[j][m] = m < nb ? wt[(size_t)(c + 4 * j) * np + 16 * m] : 0.f;
                }
#pragma unroll
                for (int j = 0; j < 4; j++)
#pragma unroll
                    for (int m = 0; m < NR; m++)
#pragma unroll
                        for (int s = 0; s < SUB; s++)
                            acc[s][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[j][s], bv[j][m], acc[s][m], 0, 0, 0);
            }
            for (; c < cpt4; c += 4) {
                float av[SUB], bv[NR];
#pragma unroll
                for (int s = 0; s < SUB; s++) av[s] = ab[s][c];
#pragma unroll
                for (int m = 0; m < NR; m++) bv[m] = m < nb ? wt[(size_t)c * np + 16 * m] : 0.f;
#pragma unroll
                for (int m = 0; m < NR; m++)
#pragma unroll
                    for (int s = 0; s < SUB; s++) acc[s][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[s], bv[m], acc[s][m], 0, 0, 0);
            }
        }
#pragma unroll
        for (int s = 0; s < SUB; s++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int q = (sg * SUB + s) * 16 + 4 * kq + r;
                if (q >= HW) continue;
#pragma unroll
                for (int m = 0; m < NR; m++) {
                    const int n = n0 + 16 * m + i16;
                    if (m >= nb || n >= N) continue;
                    float* o = out + q * so + o_off + n;
                    *o = accum ? *o + acc[s][m][r] : acc[s][m][r];
                }
            }
    }
}

// gemm_tap with NR from the column count and SUB = 2 when that still leaves every wave a unit
__device__ __forceinline__ void gemm_tap_any(const float* a, int sa, int a_off, int taps, int cpt, int d, int sgn,
                                             const float* wl, int np, float* out, int so, int o_off, int N, int H, int W,
                                             bool accum, const float* Z) {
    const int cpt4 = (cpt + 3) & ~3, nsub = (H * W + 15) >> 4;
    if (np <= 16) {
        if (nsub >= 2 * BWN)
            gemm_tap<1, 2>(a, sa, a_off, taps, cpt4, d, sgn, wl, np, out, so, o_off, N, H, W, accum, Z);
        else
            gemm_tap<1, 1>(a, sa, a_off, taps, cpt4, d, sgn, wl, np, out, so, o_off, N, H, W, accum, Z);
    } else if (np <= 32) {
        if (nsub >= 2 * BWN)
            gemm_tap<2, 2>(a, sa, a_off, taps, cpt4, d, sgn, wl, np, out, so, o_off, N, H, W, accum, Z);
        else
            gemm_tap<2, 1>(a, sa, a_off, taps, cpt4, d, sgn, wl, np, out, so, o_off, N, H, W, accum, Z);
    } else {
        gemm_tap<4, 1>(a, sa, a_off, taps, cpt4, d, sgn, wl, np, out, so, o_off, N, H, W, accum, Z);
    }
}

// dW[k][n] = sum_p A(p, k) * G[p][g_off + n] (k < K = taps * cin flat, n < N) for this image, stored to
// row[bw_map[dw + k * N + n] - lo]; with db >= 0 the bias gradient sum_p G[p][n] comes out of the same
// MFMAs as an extra row k = K of A = 1, stored to row[bw_map[db + n] - lo]. Units: (16-row k block,
// 16-column n block, pixel slice): the pixels are split into S slices when the tiles alone would
// leave waves idle, their partial tiles summed in slice order through scr (scr_floats of LDS). Pixels
// in groups of four MFMA steps: the group's A and G loads (branch-free, the row from a float
// reciprocal of W) issue together, then four MFMAs into four accumulators.
// Destinations: plain convs (direct) have the dense layout of their canonical HWIO kernel, so k * N + n
// lands at ck + k * N + n and the bias at cbias + n; the grouped branches go through bw_map (dense image
// dw / db), its entries loaded when the unit starts so their latency hides behind the MFMAs.
__device__ void wgrad_px(const float* a, int sa, int a_off, const int* kt, int K, const float* g, int sg, int g_off,
                         int N, int H, int W, const int64_t* __restrict__ bw_map, int64_t dw, int64_t db, int64_t lo,
                         float* __restrict__ row, float* scr, int scr_floats, const float* Z, bool direct = false,
                         int64_t ck = 0, int64_t cbias = 0) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i16 = lane & 15, kq = lane >> 4;
    const int HW = H * W, Kb = K + (db >= 0 ? 1 : 0), nkb = (Kb + 15) >> 4, nnb = (N + 15) >> 4, tiles = nkb * nnb;
    int S = 1;
    while (tiles * S < 2 * BWN && 2 * S * 16 <= HW && tiles * 2 * S * 256 <= scr_floats) S *= 2;
    const int q = ((HW + S - 1) / S + 15) / 16 * 16;   // pixels per slice
    const float invW = 1.f / (float)W;
    // the lane's four destinations of tile `tile` (rows k0 + 4kq + r, column n), -1: none
    auto dests = [&](int tile, int64_t (&dst)[4]) {
        const int k0 = (tile % nkb) * 16, n = (tile / nkb) * 16 + i16;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int k = k0 + 4 * kq + r;
            dst[r] = -1;
            if (n >= N) continue;
            if (k < K)
                dst[r] = direct ? ck + (int64_t)k * N + n : bw_map[dw + (int64_t)k * N + n];
            else if (k == K && db >= 0)
                dst[r] = direct ? cbias + n : bw_map[db + n];
        }
    };
    auto store = [&](const int64_t (&dst)[4], const f4& v) {
#pragma unroll
        for (int r = 0; r < 4; r++)
            if (dst[r] >= 0) row[dst[r] - lo] = v[r];
    };
    for (int unit = wave; unit < tiles * S; unit += BWN) {
        const int tile = unit % tiles, s = unit / tiles;
        const int k = (tile % nkb) * 16 + i16, n = (tile / nkb) * 16 + i16;
        const int t = k < K ? kt[k] : (k == K && db >= 0 ? KT_ONE : -1);
        int64_t dst[4];
        if (S == 1) dests(tile, dst);   // (issued before the loop: the map loads complete behind the MFMAs)
        const bool nv = n < N;
        const int p_lo = s * q, p_hi = min(HW, p_lo + q);
        f4 acc[4];
#pragma unroll
        for (int h = 0; h < 4; h++) acc[h] = f4{0.f, 0.f, 0.f, 0.f};
        for (int p0 = p_lo; p0 < p_hi; p0 += 16) {
            float av[4], bv[4];
#pragma unroll
            for (int h = 0; h < 4; h++) {
                const int p = p0 + 4 * h + kq;
                const bool pv = p < p_hi;
                const int pr = (int)(((float)p + 0.5f) * invW), pc = p - pr * W;
                av[h] = *kt_ptr(a, sa, a_off, t, pr, pc, pv, H, W, Z);
                bv[h] = *((pv && nv) ? g + p * sg + g_off + n : Z);
            }
#pragma unroll
            for (int h = 0; h < 4; h++) acc[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[h], bv[h], acc[h], 0, 0, 0);
        }
        const f4 v = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        if (S == 1)
            store(dst, v);
        else
            *reinterpret_cast<f4*>(scr + ((size_t)unit * 64 + lane) * 4) = v;
    }
    if (S > 1) {
        __syncthreads();
        for (int tile = wave; tile < tiles; tile += BWN) {
            int64_t dst[4];
            dests(tile, dst);
            f4 v = *reinterpret_cast<const f4*>(scr + ((size_t)tile * 64 + lane) * 4);
            for (int s = 1; s < S; s++) v += *reinterpret_cast<const f4*>(scr + ((size_t)(s * tiles + tile) * 64 + lane) * 4);
            store(dst, v);
        }
    }
}

// wgrad_px for images whose width is a multiple of 4, pixels walked row by row: a k-step is 4 pixels
// of one row, so the lane's A row pointer (its tap's shifted row, or Z) is set once per row and a step
// costs a pointer increment and a column bounds test instead of a table entry and a full address.
// K = taps * cin (k = tap * cin + c, the forward taps of dilation d), plus the bias row (A = 1 at ONE)
// when db >= 0; destinations, pixel slices (here: row slices) and the fixed-order slice sum as wgrad_px.
__device__ void wgrad_rows(const float* a, int sa, int a_off, int taps, int cin, int d, const float* g, int sg,
                           int g_off, int N, int H, int W, const int64_t* __restrict__ bw_map, int64_t dw, int64_t db,
                           int64_t lo, float* __restrict__ row, float* scr, int scr_floats, const float* Z,
                           const float* ONE, bool direct = false, int64_t ck = 0, int64_t cbias = 0) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i16 = lane & 15, kq = lane >> 4;
    const int K = taps * cin, Kb = K + (db >= 0 ? 1 : 0), nkb = (Kb + 15) >> 4, nnb = (N + 15) >> 4, tiles = nkb * nnb;
    int S = 1;
    while (tiles * S < 2 * BWN && 2 * S <= H && tiles * 2 * S * 256 <= scr_floats) S *= 2;
    const int q = (H + S - 1) / S;   // rows per slice
    auto dests = [&](int tile, int64_t (&dst)[4]) {
        const int k0 = (tile % nkb) * 16, n = (tile / nkb) * 16 + i16;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int k = k0 + 4 * kq + r;
            dst[r] = -1;
            if (n >= N) continue;
            if (k < K)
                dst[r] = direct ? ck + (int64_t)k * N + n : bw_map[dw + (int64_t)k * N + n];
            else if (k == K && db >= 0)
                dst[r] = direct ? cbias + n : bw_map[db + n];
        }
    };
    auto store = [&](const int64_t (&dst)[4], const f4& v) {
#pragma unroll
        for (int r = 0; r < 4; r++)
            if (dst[r] >= 0) row[dst[r] - lo] = v[r];
    };
    for (int unit = wave; unit < tiles * S; unit += BWN) {
        const int tile = unit % tiles, s = unit / tiles;
        const int k = (tile % nkb) * 16 + i16, n = (tile / nkb) * 16 + i16;
        int64_t dst[4];
        if (S == 1) dests(tile, dst);
        const bool kv = k < K, kb = k == K && db >= 0;
        const int tap = kv ? k / cin : 0, c = kv ? k - tap * cin : 0;
        const int dr = taps == 9 ? d * (tap / 3 - 1) : 0, dc = taps == 9 ? d * (tap % 3 - 1) : 0;
        const bool nv = n < N;
        const float* gcol = nv ? g + g_off + n : Z;
        const int gst = nv ? sg : 0;
        const int r_lo = s * q, r_hi = min(H, r_lo + q);
        f4 acc[4];
#pragma unroll
        for (int h = 0; h < 4; h++) acc[h] = f4{0.f, 0.f, 0.f, 0.f};
        for (int r = r_lo; r < r_hi; r++) {
            const int y = r + dr;
            const bool rv = kv && (unsigned)y < (unsigned)H;
            // the lane's A at column x: arow + x * sa (valid when rv and 0 <= x < W), the bias lane ONE
            const float* arow = a + (y * W + dc) * sa + a_off + c;
            const float* grow = gcol + (r * W + kq) * gst;
            for (int x0 = 0; x0 < W; x0 += 16) {
                float av[4], bv[4];
#pragma unroll
                for (int h = 0; h < 4; h++) {
                    const int xs = x0 + 4 * h;                 // the step's first column (uniform)
                    const bool sv = xs < W;
                    const int x = xs + kq + dc;                // the lane's source column
                    const bool in = sv && rv && (unsigned)x < (unsigned)W;
                    av[h] = *(in ? arow + (xs + kq) * sa : (kb && sv ? ONE : Z));
                    bv[h] = *(sv ? grow + xs * gst : Z);
                }
#pragma unroll
                for (int h = 0; h < 4; h++) acc[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[h], bv[h], acc[h], 0, 0, 0);
            }
        }
        const f4 v = (acc[0] + acc[1]) + (acc[2] + acc[3]);
        if (S == 1)
            store(dst, v);
        else
            *reinterpret_cast<f4*>(scr + ((size_t)unit * 64 + lane) * 4) = v;
    }
    if (S > 1) {
        __syncthreads();
        for (int tile = wave; tile < tiles; tile += BWN) {
            int64_t dst[4];
            dests(tile, dst);
            f4 v = *reinterpret_cast<const f4*>(scr + ((size_t)tile * 64 + lane) * 4);
            for (int s2 = 1; s2 < S; s2++) v += *reinterpret_cast<const f4*>(scr + ((size_t)(s2 * tiles + tile) * 64 + lane) * 4);
            store(dst, v);
        }
    }
}

// weight gradient through wgrad_rows when the width allows it, else wgrad_px over the k-table kt
// (built by the caller for K = taps * cin, cpt = cin, dilation d, sgn = +1)
__device__ __forceinline__ void wgrad_any(const float* a, int sa, int a_off, const int* kt, int taps, int cin, int d,
                                          const float* g, int sg, int g_off, int N, int H, int W,
                                          const int64_t* __restrict__ bw_map, int64_t dw, int64_t db, int64_t lo,
                                          float* __restrict__ row, float* scr, int scr_floats, const float* Z,
                                          const float* ONE, bool direct = false, int64_t ck = 0, int64_t cbias = 0) {
    if ((W & 3) == 0)
        wgrad_rows(a, sa, a_off, taps, cin, d, g, sg, g_off, N, H, W, bw_map, dw, db, lo, row, scr, scr_floats, Z, ONE,
                   direct, ck, cbias);
    else
        wgrad_px(a, sa, a_off, kt, taps * cin, g, sg, g_off, N, H, W, bw_map, dw, db, lo, row, scr, scr_floats, Z, direct,
                 ck, cbias);
}

// Wl[t * cpt4 + o][n] = W[t][n][o] (the transposed conv's B operand: dgrad of a conv with dense weights
// W[taps][cin][cout]), cpt4 = cout rounded up to 4; zero for o >= cout and n >= cin up to np columns
__device__ __forceinline__ void stage_wt(const float* __restrict__ w, int taps, int cin, int cout, int np, float* wl) {
    const int cpt4 = (cout + 3) & ~3, rows = taps * cpt4;
    const uint32_t m_np = udiv_magic(np), m_c4 = udiv_magic(cpt4);
    for (int e0 = threadIdx.x; e0 < rows * np; e0 += 4 * BWT) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int e = e0 + u * BWT;
            const int k = udiv(e, m_np), n = e - k * np;
            const int tap = udiv(k, m_c4), o = k - tap * cpt4;
            v[u] = (e < rows * np && o < cout && n < cin) ? w[((size_t)tap * cin + n) * cout + o] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; u++)
            if (e0 + u * BWT < rows * np) wl[e0 + u * BWT] = v[u];
    }
}

// fixed-order workgroup sum of two doubles (every thread gets the totals)
__device__ __forceinline__ void block_sum2(double& a, double& b, double* red) {
    a = wave_sum(a);
    b = wave_sum(b);
    if ((threadIdx.x & 63) == 0) {
        red[2 * (threadIdx.x >> 6)] = a;
        red[2 * (threadIdx.x >> 6) + 1] = b;
    }
    __syncthreads();
    double s = 0.0, t = 0.0;
#pragma unroll
    for (int w = 0; w < BWN; w++) {
        s += red[2 * w];
        t += red[2 * w + 1];
    }
    __syncthreads();   // (red reusable)
    a = s;
    b = t;
}

// LayerNorm(LeakyReLU) backward of one image (as k_lnb_reduce / k_lnb_apply): d = dL/d(LN output) in
// LDS ([HW][sd] at d_off, C channels), x the raw input (global, dense [HW][C]), gamma the per-element
// scale; dx = dL/dx to out ([HW][so] at o_off, stored or added), and the image's dgamma = d * xhat,
// dbeta = d to its row. ln == false: LeakyReLU only. Channel quads when C % 4 == 0, LU of them per
// thread with all their global loads issued before any is used (the passes are latency-bound).
constexpr int LU = 4;
__device__ void ln_bwd(const float* __restrict__ x, float mu, float rs, const float* __restrict__ gam, const float* d,
                       int sd, int d_off, float* out, int so, int o_off, bool accum, int HW, int C, bool ln,
                       float* __restrict__ rg, float* __restrict__ rb, double* red) {
    const int n = HW * C;
    const bool vq = ((C | sd | d_off | so | o_off) & 3) == 0;
    if (!ln) {
        const uint32_t m_c0 = udiv_magic(C);
        for (int e = threadIdx.x; e < n; e += BWT) {
            const int p = udiv(e, m_c0), c = e - p * C;
            const float v = d[p * sd + d_off + c] * lrelu_d(x[e]);
            float* o = out + p * so + o_off + c;
            *o = accum ? *o + v : v;
        }
        __syncthreads();
        return;
    }
    double sg = 0.0, sgh = 0.0;
    const int C4 = C >> 2, n4 = n >> 2;
    const uint32_t m_c = udiv_magic(C), m_c4 = udiv_magic(C4);
    const f4* x4 = reinterpret_cast<const f4*>(x);
    if (vq) {
        for (int i0 = threadIdx.x; i0 < n4; i0 += LU * BWT) {
            f4 xv[LU], gv[LU];
#pragma unroll
            for (int u = 0; u < LU; u++) {
                const int i = i0 + u * BWT;
                xv[u] = i < n4 ? x4[i] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < 4; j++) gv[u][j] = i < n4 ? gam[4 * i + j] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < LU; u++) {
                const int i = i0 + u * BWT;
                if (i >= n4) break;
                const int p = udiv(i, m_c4), c = (i - p * C4) << 2;
                const f4 dv = *reinterpret_cast<const f4*>(d + p * sd + d_off + c);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float xh = (lrelu_b(xv[u][j]) - mu) * rs;
                    const float g = dv[j] * gv[u][j];
                    sg += g;
                    sgh += (double)g * xh;
                }
            }
        }
    } else {
        for (int e = threadIdx.x; e < n; e += BWT) {
            const int p = udiv(e, m_c), c = e - p * C;
            const float xh = (lrelu_b(x[e]) - mu) * rs;
            const float g = d[p * sd + d_off + c] * gam[e];
            sg += g;
            sgh += (double)g * xh;
        }
    }
    block_sum2(sg, sgh, red);
    const float inv_n = 1.f / (float)n;
    const float mg = (float)(sg * inv_n), mgh = (float)(sgh * inv_n);
    if (vq) {
        for (int i0 = threadIdx.x; i0 < n4; i0 += LU * BWT) {
            f4 xv[LU], gv[LU];
#pragma unroll
            for (int u = 0; u < LU; u++) {
                const int i = i0 + u * BWT;
                xv[u] = i < n4 ? x4[i] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < 4; j++) gv[u][j] = i < n4 ? gam[4 * i + j] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < LU; u++) {
                const int i = i0 + u * BWT;
                if (i >= n4) break;
                const int p = udiv(i, m_c4), c = (i - p * C4) << 2;
                const f4 dv = *reinterpret_cast<const f4*>(d + p * sd + d_off + c);
                f4* o = reinterpret_cast<f4*>(out + p * so + o_off + c);
                f4 ov = accum ? *o : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float xh = (lrelu_b(xv[u][j]) - mu) * rs;
                    rg[4 * i + j] = dv[j] * xh;
                    rb[4 * i + j] = dv[j];
                    ov[j] += rs * (dv[j] * gv[u][j] - mg - xh * mgh) * lrelu_d(xv[u][j]);
                }
                *o = ov;
            }
        }
    } else {
        for (int e = threadIdx.x; e < n; e += BWT) {
            const int p = udiv(e, m_c), c = e - p * C;
            const float xv = x[e];
            const float xh = (lrelu_b(xv) - mu) * rs;
            const float dv = d[p * sd + d_off + c];
            rg[e] = dv * xh;
            rb[e] = dv;
            const float v = rs * (dv * gam[e] - mg - xh * mgh) * lrelu_d(xv);
            float* o = out + p * so + o_off + c;
            *o = accum ? *o + v : v;
        }
    }
    __syncthreads();
}

// stage LN(LeakyReLU(x)) (or LeakyReLU(x) when !ln) of channels [c0, c0 + nc) of a C-channel raw tensor
// x (global, dense) into dst [HW][sd] from channel 0
__device__ void stage_act(const float* __restrict__ x, int C, int c0, int nc, int HW, float mu, float rs,
                          const float* __restrict__ gam, const float* __restrict__ bet, bool ln, float* dst, int sd) {
    if (((C | c0 | nc | sd) & 3) == 0) {
        const int nq = nc >> 2, n4 = HW * nq;
        const uint32_t m_nq = udiv_magic(nq);
        for (int i0 = threadIdx.x; i0 < n4; i0 += LU * BWT) {
            f4 xv[LU], gv[LU], bv[LU];
#pragma unroll
            for (int u = 0; u < LU; u++) {
                const int i = i0 + u * BWT;
                const int p = udiv(i, m_nq), c = (i - p * nq) << 2;
                const size_t gi = (size_t)p * C + c0 + c;
                xv[u] = i < n4 ? *reinterpret_cast<const f4*>(x + gi) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    gv[u][j] = (ln && i < n4) ? gam[gi + j] : 0.f;
                    bv[u][j] = (ln && i < n4) ? bet[gi + j] : 0.f;
                }
            }
#pragma unroll
            for (int u = 0; u < LU; u++) {
                const int i = i0 + u * BWT;
                if (i >= n4) break;
                const int p = udiv(i, m_nq), c = (i - p * nq) << 2;
                f4 v;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float h = lrelu_b(xv[u][j]);
                    v[j] = ln ? (h - mu) * rs * gv[u][j] + bv[u][j] : h;
                }
                *reinterpret_cast<f4*>(dst + p * sd + c) = v;
            }
        }
        return;
    }
    const int n = HW * nc;
    const uint32_t m_nc = udiv_magic(nc);
    for (int e = threadIdx.x; e < n; e += BWT) {
        const int p = udiv(e, m_nc), c = e - p * nc;
        const size_t gi = (size_t)p * C + c0 + c;
        const float h = lrelu_b(x[gi]);
        dst[p * sd + c] = ln ? (h - mu) * rs * gam[gi] + bet[gi] : h;
    }
}

// dst[p * C + c] = src[p * ss + c] (LDS -> global, dense) and back; C % 4 == 0 and ss % 4 == 0 take quads
__device__ void store_lds(float* __restrict__ dst, const float* src, int ss, int HW, int C) {
    if (((C | ss) & 3) == 0) {
        const int cq = C >> 2, n = HW * cq;
        const uint32_t m = udiv_magic(cq);
        for (int i = threadIdx.x; i < n; i += BWT) {
            const int p = udiv(i, m), c = (i - p * cq) << 2;
            *reinterpret_cast<f4*>(dst + (size_t)p * C + c) = *reinterpret_cast<const f4*>(src + p * ss + c);
        }
        return;
    }
    const uint32_t m = udiv_magic(C);
    for (int i = threadIdx.x; i < HW * C; i += BWT) {
        const int p = udiv(i, m), c = i - p * C;
        dst[i] = src[p * ss + c];
    }
}
__device__ void load_lds(float* dst, int ss, const float* __restrict__ src, int HW, int C) {
    if (((C | ss) & 3) == 0) {
        const int cq = C >> 2, n = HW * cq;
        const uint32_t m = udiv_magic(cq);
        for (int i0 = threadIdx.x; i0 < n; i0 += 4 * BWT) {
            f4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = min(i0 + u * BWT, n - 1);
                const int p = udiv(i, m), c = (i - p * cq) << 2;
                v[u] = *reinterpret_cast<const f4*>(src + (size_t)p * C + c);
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int i = i0 + u * BWT;
                if (i >= n) break;
                const int p = udiv(i, m), c = (i - p * cq) << 2;
                *reinterpret_cast<f4*>(dst + p * ss + c) = v[u];
            }
        }
        return;
    }
    const uint32_t m = udiv_magic(C);
    for (int i = threadIdx.x; i < HW * C; i += BWT) {
        const int p = udiv(i, m), c = i - p * C;
        dst[p * ss + c] = src[i];
    }
}

// position in u of element (pixel p, channel c) of the mask-compressed u1c (mask compress, :720-759)
__device__ __forceinline__ int mask_pos_b(int m, int p, int c, int wc, int W, int D) {
    const int pr = p / wc, pc = p - pr * wc;
    if (m < 2) {
        const int half = c >= D ? 1 : 0;
        const int ch = c - half * D;
        const int dcol = (m == 0) ? half : 1 - half;
        return ((2 * pr + half) * W + (2 * pc + dcol)) * D + ch;
    }
    return (pr * W + pc) * D + ((m == 2) ? 2 * c : 2 * c + 1);
}

}  // namespace

// diagnostics (LdsBwdArgs::stamps != 0): thread 0 of workgroup (0, 0) records the shader clock at every
// phase boundary of the last k_lds_bwd launch (cnf_debug_read_bwd_stamps)
__device__ long long g_bwd_stamps[128];
#define BSTAMP()                                                                                     \
    do {                                                                                              \
        if (a.stamps && threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0 && nst < 127)          \
            g_bwd_stamps[1 + nst++] = (long long)__builtin_amdgcn_s_memtime();                         \
    } while (0)

// offsets table per net (LdsBwdArgs::offs): see LDSBWD_* in cnf_kernels.h
__global__ __launch_bounds__(BWT) void k_lds_bwd(LdsBwdArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int img = blockIdx.x, net = blockIdx.y, B = gridDim.x;
    const int H = a.hc, W = a.wc, HW = H * W, nk = a.nk, gc = a.gc, R = a.R;
    const bool ln = a.ln != 0;
    float* GY = reinterpret_cast<float*>(smem);
    float* GT = reinterpret_cast<float*>(smem + a.off_gt);
    float* AC = reinterpret_cast<float*>(smem + a.off_ac);
    float* WL = reinterpret_cast<float*>(smem + a.off_w);
    int* KT = reinterpret_cast<int*>(smem + a.off_kt);
    double* RED = reinterpret_cast<double*>(smem + a.off_red);
    int* OT = reinterpret_cast<int*>(smem + a.off_ot);
    float* ZQ = reinterpret_cast<float*>(smem + a.off_z);   // 4 zeros, then 4 ones (kt_ptr, wgrad_rows)
    const float* ZR = ZQ + 8;                                  // a.zn zeros: gemm_tap's row outside the image
    // zero the whole LDS image once: gemm_tap's padded channels read A values next to their windows, which
    // must be finite
    for (int i = threadIdx.x; i < (a.lds_bytes >> 4); i += BWT)
        reinterpret_cast<f4*>(smem)[i] = f4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
    if (threadIdx.x < 8) ZQ[threadIdx.x] = threadIdx.x < 4 ? 0.f : 1.f;
    const int SY = a.sy, ST = a.st, SA = a.sa;
    int nst = 0;
    BSTAMP();
    for (int i = threadIdx.x; i < a.offs_per_net; i += BWT) OT[i] = a.offs[net * a.offs_per_net + i];
    __syncthreads();
        BSTAMP();
    const int64_t lo = OT[LDSBWD_LO];
    const float* sv = a.save + ((size_t)net * B + img) * a.save_img;
    const float* st = sv + a.save_st;
    const float* P = a.params;
    const float* BWI = a.bw;
    float* row = a.part + ((size_t)net * B + img) * a.row;
    auto rbo = [&](int r) { return OT + LDSBWD_RB0 + r * (LDSBWD_PER_RB0 + 2 * a.nbr); };
    auto kp4 = [](int K) { return (K + 3) & ~3; };
    auto np16 = [](int N) { return (N + 15) & ~15; };
    const int taps = a.taps;
    const uint32_t m_nk = udiv_magic(nk);
    // split mode: CH = the data-gradient chain (+ LN gamma / beta rows), WG = the weight gradients; mode 1
    // stores the gradients each weight gradient contracts with, mode 2 reads them back (a.gsave)
    const bool CH = a.mode != 2, WG = a.mode != 1, store = a.mode == 1, load = a.mode == 2;
    float* gs = a.gsave ? a.gsave + ((size_t)net * B + img) * a.gsave_img : nullptr;
    if (CH && OT[LDSBWD_TANH] >= 0 && threadIdx.x == 0) row[OT[LDSBWD_TANH] - lo] = 0.f;   // (k_dsum adds it)

    // ---- conv_out: G = dL/d so (dc2 ch) -> GT; A = LN_out(y_R) -> AC; wgrad; dgrad -> GY
    {
        const float* ds = a.dso[net] + (size_t)img * HW * a.dc2;
        const uint32_t m_d2 = udiv_magic(a.dc2);
        for (int e = threadIdx.x; e < HW * a.dc2; e += BWT) {
            const int p = udiv(e, m_d2), c = e - p * a.dc2;
            GT[p * ST + c] = ds[e];
        }
        const float* yR = sv + (size_t)R * HW * nk;
        const float mu = st[6 * R], rs = st[6 * R + 1];
        if (WG) {
            stage_act(yR, nk, 0, nk, HW, mu, rs, ln ? P + OT[LDSBWD_LNO_G] : nullptr,
                      ln ? P + OT[LDSBWD_LNO_B] : nullptr, ln, AC, SA);
            build_kt(KT, taps * nk, kp4(taps * nk), nk, taps, 1, 1);
            __syncthreads();
            BSTAMP();
            wgrad_any(AC, SA, 0, KT, taps, nk, 1, GT, ST, 0, a.dc2, H, W, a.bw_map, OT[LDSBWD_CO_DW], OT[LDSBWD_CO_DB], lo,
                      row, WL, a.wmax, ZQ, ZQ + 4, true, OT[LDSBWD_CO_K], OT[LDSBWD_CO_B]);
            __syncthreads();
            BSTAMP();
        }
        if (CH) {
            stage_wt(BWI + OT[LDSBWD_CO_DW], taps, nk, a.dc2, np16(nk), WL);
            __syncthreads();
            BSTAMP();
            gemm_tap_any(GT, ST, 0, taps, a.dc2, 1, -1, WL, np16(nk), GY, SY, 0, nk, H, W, false, ZR);
            __syncthreads();
            BSTAMP();
            // LN_out backward in place on GY
            ln_bwd(yR, mu, rs, ln ? P + OT[LDSBWD_LNO_G] : nullptr, GY, SY, 0, GY, SY, 0, false, HW, nk, ln,
                   ln ? row + (OT[LDSBWD_LNO_G] - lo) : nullptr, ln ? row + (OT[LDSBWD_LNO_B] - lo) : nullptr, RED);
            BSTAMP();
        }
    }
    for (int r = R - 1; r >= 0; r--) {
        const int* o = rbo(r);
        const float* yr = sv + (size_t)r * HW * nk;
        const float* t1r = sv + a.save_t1 + (size_t)r * HW * nk;
        const float* t2r = sv + a.save_t2 + (size_t)r * HW * gc;
        const float mu1 = st[2 * r], rs1 = st[2 * r + 1];
        const float mu2 = st[2 * (R + r)], rs2 = st[2 * (R + r) + 1];
        const float mu3 = st[2 * (2 * R + r)], rs3 = st[2 * (2 * R + r) + 1];
        float* gr = gs ? gs + (size_t)r * a.gs_rb : nullptr;
        if (store) store_lds(gr, GY, SY, HW, nk);   // dL/dy_{r+1}: conv_b's weight gradient
        if (load) {
            load_lds(GY, SY, gr, HW, nk);
            __syncthreads();
        }
        // ---- conv_b (y_{r+1} = y_r + conv_b(LN3(t2_r))): wgrad in channel chunks of the staged LN3(t2),
        // dgrad dL/d LN3-out -> GT
        if (WG)
            for (int c0 = 0; c0 < gc; c0 += a.ac_chunk) {
                const int nc = gc - c0 < a.ac_chunk ? gc - c0 : a.ac_chunk;
                stage_act(t2r, gc, c0, nc, HW, mu3, rs3, ln ? P + o[LDSBWD_LN3G] : nullptr,
                          ln ? P + o[LDSBWD_LN3B] : nullptr, ln, AC, SA);
                build_kt(KT, nc, kp4(nc), nc, 1, 1, 1);
                __syncthreads();
                BSTAMP();
                // rows c0.. of conv_b's dense [gc][nk] image: offset the dense base by c0 * nk (the bias
                // gradient once, with the first chunk)
                wgrad_any(AC, SA, 0, KT, 1, nc, 1, GY, SY, 0, nk, H, W, a.bw_map, o[LDSBWD_CB_DW] + (int64_t)c0 * nk,
                          c0 == 0 ? (int64_t)o[LDSBWD_CB_DB] : -1, lo, row, WL, a.wmax, ZQ, ZQ + 4, true,
                          o[LDSBWD_CB_K] + (int64_t)c0 * nk, o[LDSBWD_CB_B]);
                __syncthreads();
                BSTAMP();
            }
        if (CH) {
            stage_wt(BWI + o[LDSBWD_CB_DW], 1, gc, nk, np16(gc), WL);
            __syncthreads();
            BSTAMP();
            gemm_tap_any(GY, SY, 0, 1, nk, 1, -1, WL, np16(gc), GT, ST, 0, gc, H, W, false, ZR);
            __syncthreads();
            BSTAMP();
            // ---- LN3 backward in place on GT -> dL/dt2
            ln_bwd(t2r, mu3, rs3, ln ? P + o[LDSBWD_LN3G] : nullptr, GT, ST, 0, GT, ST, 0, false, HW, gc, ln,
                   ln ? row + (o[LDSBWD_LN3G] - lo) : nullptr, ln ? row + (o[LDSBWD_LN3B] - lo) : nullptr, RED);
            BSTAMP();
        }
        if (store) store_lds(gr + a.g_t3, GT, ST, HW, gc);   // dL/dt2: the branches' weight gradients
        if (load) {
            load_lds(GT, ST, gr + a.g_t3, HW, gc);
            __syncthreads();
        }
        // ---- grouped branches: every wgrad (A = LN2(t1) window -> AC), then every dgrad into AC (zeroed)
        if (WG)
            for (int bi = 0; bi < a.nbr; bi++) {
                const int cin = a.br_cin[bi], cout = a.br_cout[bi];
                stage_act(t1r, nk, a.br_cin_off[bi], cin, HW, mu2, rs2, ln ? P + o[LDSBWD_LN2G] : nullptr,
                          ln ? P + o[LDSBWD_LN2B] : nullptr, ln, AC, SA);
                build_kt(KT, taps * cin, kp4(taps * cin), cin, taps, a.br_dil[bi], 1);
                __syncthreads();
                BSTAMP();
                wgrad_any(AC, SA, 0, KT, taps, cin, a.br_dil[bi], GT, ST, a.br_out_off[bi], cout, H, W, a.bw_map,
                          o[LDSBWD_BR + 2 * bi], o[LDSBWD_BR + 2 * bi + 1], lo, row, WL, a.wmax, ZQ, ZQ + 4);
                __syncthreads();
                BSTAMP();
            }
        if (CH) {
            for (int e = threadIdx.x; e < HW * nk; e += BWT) {
                const int p = udiv(e, m_nk), c = e - p * nk;
                AC[p * SA + c] = 0.f;
            }
            for (int bi = 0; bi < a.nbr; bi++) {
                const int cin = a.br_cin[bi], cout = a.br_cout[bi];
                stage_wt(BWI + o[LDSBWD_BR + 2 * bi], taps, cin, cout, np16(cin), WL);
                __syncthreads();
                BSTAMP();
                gemm_tap_any(GT, ST, a.br_out_off[bi], taps, cout, a.br_dil[bi], -1, WL, np16(cin), AC, SA, a.br_cin_off[bi],
                             cin, H, W, true, ZR);
                __syncthreads();
                BSTAMP();
            }
            // ---- LN2 backward: AC (dL/d LN2-out, zero outside the windows) -> dL/dt1 in GT
            ln_bwd(t1r, mu2, rs2, ln ? P + o[LDSBWD_LN2G] : nullptr, AC, SA, 0, GT, ST, 0, false, HW, nk, ln,
                   ln ? row + (o[LDSBWD_LN2G] - lo) : nullptr, ln ? row + (o[LDSBWD_LN2B] - lo) : nullptr, RED);
            BSTAMP();
        }
        if (store) store_lds(gr + a.g_t2, GT, ST, HW, nk);   // dL/dt1: conv_a's weight gradient
        if (load) {
            load_lds(GT, ST, gr + a.g_t2, HW, nk);
            __syncthreads();
        }
        // ---- conv_a: A = LN1(y_r) -> AC; wgrad with GT; dgrad -> AC
        if (WG) {
            stage_act(yr, nk, 0, nk, HW, mu1, rs1, ln ? P + o[LDSBWD_LN1G] : nullptr, ln ? P + o[LDSBWD_LN1B] : nullptr,
                      ln, AC, SA);
            build_kt(KT, nk, kp4(nk), nk, 1, 1, 1);
            __syncthreads();
            BSTAMP();
            wgrad_any(AC, SA, 0, KT, 1, nk, 1, GT, ST, 0, nk, H, W, a.bw_map, o[LDSBWD_CA_DW], o[LDSBWD_CA_DB], lo, row,
                      WL, a.wmax, ZQ, ZQ + 4, true, o[LDSBWD_CA_K], o[LDSBWD_CA_B]);
            __syncthreads();
            BSTAMP();
        }
        if (CH) {
            stage_wt(BWI + o[LDSBWD_CA_DW], 1, nk, nk, np16(nk), WL);
            __syncthreads();
            BSTAMP();
            gemm_tap_any(GT, ST, 0, 1, nk, 1, -1, WL, np16(nk), AC, SA, 0, nk, H, W, false, ZR);
            __syncthreads();
            BSTAMP();
            // ---- LN1 backward: GY += dL/dy_r through conv_a (the identity path keeps GY)
            ln_bwd(yr, mu1, rs1, ln ? P + o[LDSBWD_LN1G] : nullptr, AC, SA, 0, GY, SY, 0, true, HW, nk, ln,
                   ln ? row + (o[LDSBWD_LN1G] - lo) : nullptr, ln ? row + (o[LDSBWD_LN1B] - lo) : nullptr, RED);
            BSTAMP();
        }
    }
    // ---- conv_in: A = u1c (gathered from the layer input) -> AC; wgrad with GY; dgrad -> GT -> du1c
    {
        if (store) store_lds(gs + a.g_in, GY, SY, HW, nk);   // dL/dy_0: conv_in's weight gradient
        if (load) {
            load_lds(GY, SY, gs + a.g_in, HW, nk);
            __syncthreads();
        }
        const uint32_t m_d1 = udiv_magic(a.dc1);
        if (WG) {
            const float* ub = a.u + (size_t)img * a.H * a.W * a.D;
            for (int e = threadIdx.x; e < HW * a.dc1; e += BWT) {
                const int p = udiv(e, m_d1), c = e - p * a.dc1;
                AC[p * SA + c] = ub[mask_pos_b(a.mask, p, c, W, a.W, a.D)];
            }
            build_kt(KT, taps * a.dc1, kp4(taps * a.dc1), a.dc1, taps, 1, 1);
            __syncthreads();
            BSTAMP();
            wgrad_any(AC, SA, 0, KT, taps, a.dc1, 1, GY, SY, 0, nk, H, W, a.bw_map, OT[LDSBWD_CI_DW], OT[LDSBWD_CI_DB], lo,
                      row, WL, a.wmax, ZQ, ZQ + 4, true, OT[LDSBWD_CI_K], OT[LDSBWD_CI_B]);
            __syncthreads();
            BSTAMP();
        }
        if (CH) {
            stage_wt(BWI + OT[LDSBWD_CI_DW], taps, a.dc1, nk, np16(a.dc1), WL);
            __syncthreads();
            BSTAMP();
            gemm_tap_any(GY, SY, 0, taps, nk, 1, -1, WL, np16(a.dc1), GT, ST, 0, a.dc1, H, W, false, ZR);
            __syncthreads();
            BSTAMP();
            float* du = a.du1c[net] + (size_t)img * HW * a.dc1;
            for (int e = threadIdx.x; e < HW * a.dc1; e += BWT) {
                const int p = udiv(e, m_d1), c = e - p * a.dc1;
                du[e] = GT[p * ST + c];
            }
        }
    }
    BSTAMP();
    if (a.stamps && threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) g_bwd_stamps[0] = nst;
}

int read_bwd_stamps(long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_bwd_stamps), sizeof(long long) * (n > 128 ? 128 : n)) == hipSuccess ? 0
                                                                                                                   : -1;
}

void launch_lds_bwd(const LdsBwdArgs& a, int B, hipStream_t st) {
    hipLaunchKernelGGL(k_lds_bwd, dim3(B, 2), dim3(BWT), a.lds_bytes, st, a);
}

// dst[net][i] += sum over images b of part[net][b][i], i < row; lo[net]: the net's first canonical
// parameter. 32 elements per workgroup, 8 image slices per element (slice s: images s, s + 8, ...,
// all of them in flight at once up to B = 64), fp64 sums, then a fixed-order LDS sum over the
// slices: deterministic
constexpr int GR_EL = 32, GR_SL = 8, GR_U = 8;
__global__ __launch_bounds__(GR_EL * GR_SL) void k_grad_rows(const float* __restrict__ part, int B, int row, int64_t lo0,
                                                             int64_t lo1, int len0, int len1, float* __restrict__ dparams) {
    __shared__ double red[GR_SL][GR_EL];
    const int net = blockIdx.y;
    const int el = threadIdx.x & (GR_EL - 1), sl = threadIdx.x / GR_EL;
    const int i = blockIdx.x * GR_EL + el;
    const int len = net == 0 ? len0 : len1;
    const float* pr = part + (size_t)net * B * row + i;
    float old = 0.f;
    float* d = dparams + (net == 0 ? lo0 : lo1) + i;
    if (sl == 0 && i < len) old = *d;
    double s = 0.0;
    if (i < len) {
        for (int b0 = sl; b0 < B; b0 += GR_SL * GR_U) {
            float v[GR_U];
#pragma unroll
            for (int u = 0; u < GR_U; u++) {
                const int b = b0 + GR_SL * u;
                v[u] = b < B ? pr[(size_t)b * row] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < GR_U; u++) s += (double)v[u];
        }
    }
    red[sl][el] = s;
    __syncthreads();
    if (sl == 0 && i < len) {
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < GR_SL; k++) tot += red[k][el];
        *d = old + (float)tot;
    }
}

void launch_grad_rows(const float* part, int B, int row, int64_t lo0, int64_t lo1, int len0, int len1, float* dparams,
                      hipStream_t st) {
    const int n = len0 > len1 ? len0 : len1;
    hipLaunchKernelGGL(k_grad_rows, dim3((n + GR_EL - 1) / GR_EL, 2), dim3(GR_EL * GR_SL), 0, st, part, B, row, lo0, lo1,
                       len0, len1, dparams);
}

}  // namespace cnf
