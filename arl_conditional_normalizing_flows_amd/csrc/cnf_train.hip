// cnf_train.hip — kernels of the NLL training step (cFlow.train_step, conv_cINN_make_model.py:1850-1880:
// GradientTape over log_loss, then Adam).
//
// The backward pass recomputes each coupling layer's s,t networks from the layer's saved input and
// walks them in reverse. Every convolution of the forward recompute, the data gradient (conv^T) and
// the weight gradient runs on the dense backward image (taps x cin x cout per conv, cnf_plan.h),
// so the training path is independent of the inference kernels' packed LDS formats:
//   k_tconv      register-blocked (4 px x 4 ch per lane) LDS-tiled fp32 conv, forward or transposed,
//                LN + LeakyReLU applied on load, bias / residual / accumulate in the epilogue
//   k_wgrad      per-chunk outer-product sums X^T dY (LN-on-load), 64 x 64 (ci, co) tiles
//   k_grad_scatter  chunk reduction + scatter onto the canonical parameters through the dense map
//   k_ln_stats / k_lnb_reduce / k_lnb_apply   LayerNorm(LeakyReLU) backward, per image, with the
//                per-element gamma/beta gradients accumulated over the batch in registers
//   k_coup_bw    affine coupling law backward (exp / tanh scale / log-det term)
//   k_adam       Keras Adam update
// fp32 storage, fp64 for every per-image reduction.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <algorithm>
#include <cstdlib>
#include <stdexcept>

#include "cnf_device.h"
#include "cnf_kernels.h"

namespace cnf {

namespace {

__device__ __forceinline__ float act_load(float x, int act, const float* stats, const float* gamma, const float* beta,
                                          int b, size_t gi) {
    if (stats) {
        const float h = lrelu(x);
        return (h - stats[2 * b]) * stats[2 * b + 1] * gamma[gi] + beta[gi];
    }
    return act ? lrelu(x) : x;
}

__device__ __forceinline__ double block_sum256(double v, double* red) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    return red[0] + red[1] + red[2] + red[3];
}

}  // namespace

// ------------------------------------------------------------------------------------------------
// k_tconv: tile = TP pixels (row-major run inside one image) x TN output channels; each of the 256
// lanes owns 4 pixels x 4 channels. K is consumed in chunks of KC channels per tap.
// ------------------------------------------------------------------------------------------------
template <int TN>
__global__ __launch_bounds__(256) void k_tconv(TConvArgs a) {
    constexpr int TP = 4096 / TN;              // 64 / 256 / 1024 pixels
    constexpr int KC = TN == 64 ? 16 : TN == 16 ? 8 : 4;
    constexpr int XS = TP + 4;                 // LDS row stride (16-byte aligned)
    __shared__ __attribute__((aligned(16))) float Xs[KC * XS];
    __shared__ __attribute__((aligned(16))) float Ws[KC * TN];
    const int t = threadIdx.x;
    const int tx = t % (TP / 4), ty = t / (TP / 4);
    const int npx = a.H * a.W;
    const int b = blockIdx.y;
    const int p0 = blockIdx.x * TP, n0 = blockIdx.z * TN;
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = 0.f;
    const float* inb = a.in + (size_t)b * npx * a.in_cs + a.in_off;
    for (int tap = 0; tap < a.taps; tap++) {
        const int dr = a.taps == 1 ? 0 : tap / 3 - 1, dc = a.taps == 1 ? 0 : tap % 3 - 1;
        const int sr = a.sgn * a.dil * dr, sc = a.sgn * a.dil * dc;
        for (int k0 = 0; k0 < a.K; k0 += KC) {
            // stage X: KC channels (fastest) x TP pixels
            for (int e = t; e < KC * TP; e += 256) {
                const int k = e % KC, px = e / KC;
                const int p = p0 + px;
                float v = 0.f;
                if (p < npx && k0 + k < a.K) {
                    const int r = p / a.W + sr, c = p % a.W + sc;
                    if (r >= 0 && r < a.H && c >= 0 && c < a.W) {
                        const size_t q = (size_t)r * a.W + c;
                        v = act_load(inb[q * a.in_cs + k0 + k], a.act, a.stats, a.gamma, a.beta, b,
                                     q * a.in_cs + a.in_off + k0 + k);
                    }
                }
                Xs[k * XS + px] = v;
            }
            for (int e = t; e < KC * TN; e += 256) {
                const int n = e % TN, k = e / TN;
                float v = 0.f;
                if (k0 + k < a.K && n0 + n < a.N) v = a.w[tap * a.wt + (long long)(k0 + k) * a.wk + (long long)(n0 + n) * a.wn];
                Ws[k * TN + n] = v;
            }
            __syncthreads();
#pragma unroll
            for (int k = 0; k < KC; k++) {
                const f4 x = *reinterpret_cast<const f4*>(&Xs[k * XS + 4 * tx]);
                const f4 w = *reinterpret_cast<const f4*>(&Ws[k * TN + 4 * ty]);
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 4; j++) acc[i][j] = fmaf(x[i], w[j], acc[i][j]);
            }
            __syncthreads();
        }
    }
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int p = p0 + 4 * tx + i;
        if (p >= npx) continue;
        const size_t ob = ((size_t)b * npx + p) * a.out_cs + a.out_off;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int n = n0 + 4 * ty + j;
            if (n >= a.N) continue;
            float v = acc[i][j];
            if (a.bias) v += a.bias[n];
            if (a.res) v += a.res[ob + n];
            if (a.accumulate) v += a.out[ob + n];
            a.out[ob + n] = v;
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_tconv_mfma: the same convolution as an implicit GEMM on v_mfma_f32_16x16x4_f32. A workgroup of
// 4 waves owns 64 pixels (16 per wave) x 16*NR output channels of one image. Per tap, the weights
// W(tap, k, n) are staged into LDS as [g][kq][j][s] (k = 16g + 4kq + s, j = n - n0), so lane (i16, kq)
// reads one float4 per 16-column block; its A operand is the float4 of channels 16g + 4kq .. +3 of
// its (shifted) pixel, loaded straight from global with LN + LeakyReLU applied in registers. The
// K order inside a group is permuted identically on both operands, so the sum is the conv's.
// ------------------------------------------------------------------------------------------------
// fused LN-backward reduction (TConvArgs::lnr_part): the workgroup's (sum g, sum g * xhat), fixed order
__device__ __forceinline__ void lnr_finish(const TConvArgs& a, double sg, double sgh, int b) {
    __shared__ double lred[8];
    sg = wave_sum(sg);
    sgh = wave_sum(sgh);
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    __syncthreads();   // (the kernel's LDS reads are done; lred is static, disjoint anyway)
    if (lane == 0) {
        lred[2 * wave] = sg;
        lred[2 * wave + 1] = sgh;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double s0 = 0.0, s1 = 0.0;
        for (int w = 0; w < 4; w++) {
            s0 += lred[2 * w];
            s1 += lred[2 * w + 1];
        }
        const size_t k = (size_t)b * a.lnr_stride + a.lnr_base + blockIdx.x + gridDim.x * blockIdx.z;
        a.lnr_part[2 * k] = s0;
        a.lnr_part[2 * k + 1] = s1;
    }
}
#ifndef CNF_TW_U
#define CNF_TW_U 8
#endif
constexpr int TW_U = CNF_TW_U;   // weight-staging loads in flight per thread

template <int NR, bool VEC>
__global__ __launch_bounds__(256) void k_tconv_mfma(TConvArgs a, int all_taps) {
    extern __shared__ __attribute__((aligned(16))) float wsm[];
    constexpr int NS = 16 * NR;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i16 = lane & 15, kq = lane >> 4;
    const int npx = a.H * a.W, b = blockIdx.y;
    const int p0 = blockIdx.x * 64, n0 = blockIdx.z * NS;
    const int G = (a.K + 15) >> 4;
    const int pa = p0 + wave * 16 + i16;
    const bool pav = pa < npx;
    const int pr = pa / a.W, pc = pa - pr * a.W;
    const float* inb = a.in + (size_t)b * npx * a.in_cs + a.in_off;
    const bool ln = a.stats != nullptr;
    const float mu = ln ? a.stats[2 * b] : 0.f, rs = ln ? a.stats[2 * b + 1] : 1.f;
    const uint32_t inbytes = (uint32_t)(npx * a.in_cs - a.in_off) * 4u;
    const __amdgpu_buffer_rsrc_t rin = buf_rsrc(inb, inbytes);
    const __amdgpu_buffer_rsrc_t rgm = buf_rsrc(ln ? a.gamma + a.in_off : inb, inbytes);
    const __amdgpu_buffer_rsrc_t rbt = buf_rsrc(ln ? a.beta + a.in_off : inb, inbytes);
    f4 acc[NR];
#pragma unroll
    for (int m = 0; m < NR; m++) acc[m] = f4{0.f, 0.f, 0.f, 0.f};
    const int nw = G * 16 * NS;   // weight floats of one tap
    // (TW_U loads in flight per thread: the transposed weight reads are scattered 4-byte loads, and one
    // at a time they cost a memory round trip each)
    const bool wvec = a.wk == 1 && (a.wn & 3) == 0 && (a.K & 3) == 0 && a.wt * a.taps < (1LL << 29);
    const __amdgpu_buffer_rsrc_t rw = buf_rsrc(a.w, (uint32_t)((a.wt * a.taps) * 4));
    auto stage_w = [&](int tap, float* dst) {
        if (wvec) {   // (as in k_tconv_band: one 16-byte load per (gq, j) of a data gradient's weights)
            const int nw4 = nw >> 2;
            for (int e0 = threadIdx.x; e0 < nw4; e0 += 256 * TW_U) {
                f4 v[TW_U];
#pragma unroll
                for (int u = 0; u < TW_U; u++) {
                    const int e = e0 + 256 * u;
                    const int j = e % NS, gq = e / NS;
                    const int k = 4 * gq, n = n0 + j;
                    const bool ok = e < nw4 && k < a.K && n < a.N;
                    v[u] = buf_load4(rw, ok ? (uint32_t)(tap * (int)a.wt + n * a.wn + k) * 4u : BUF_OOB);
                }
#pragma unroll
                for (int u = 0; u < TW_U; u++)
                    if (e0 + 256 * u < nw4) *reinterpret_cast<f4*>(dst + 4 * (e0 + 256 * u)) = v[u];
            }
            return;
        }
        for (int e0 = threadIdx.x; e0 < nw; e0 += 256 * TW_U) {
            float v[TW_U];
#pragma unroll
            for (int u = 0; u < TW_U; u++) {
                const int e = e0 + 256 * u;
                const int s4 = e & 3, j = (e >> 2) % NS, gq = (e >> 2) / NS;   // gq = 4g + kq'
                const int k = 4 * gq + s4, n = n0 + j;
                const bool ok = e < nw && k < a.K && n < a.N;
                v[u] = *(ok ? a.w + (tap * a.wt + (long long)k * a.wk + (long long)n * a.wn) : a.zero);
            }
#pragma unroll
            for (int u = 0; u < TW_U; u++)
                if (e0 + 256 * u < nw) dst[e0 + 256 * u] = v[u];
        }
    };
    // A operand of flat step it = tap * G + g: raw channels 16g + 4kq .. +3 of the lane's shifted pixel
    // (+ its LN gamma / beta), loaded one step ahead so the loads overlap the previous step's MFMAs
    auto load = [&](int tap, int g, f4& x, f4& gm, f4& bt) -> bool {
        const int dr = a.taps == 1 ? 0 : tap / 3 - 1, dc = a.taps == 1 ? 0 : tap % 3 - 1;
        const int r = pr + a.sgn * a.dil * dr, c = pc + a.sgn * a.dil * dc;
        const int k0 = 16 * g + 4 * kq;
        const bool sv = pav && r >= 0 && r < a.H && c >= 0 && c < a.W && k0 < a.K;
        const size_t gi = ((size_t)r * a.W + c) * a.in_cs + k0;
        if (VEC) {   // branch-free buffer loads: an invalid lane's offset is out of range and reads zeros
            const uint32_t off = sv ? (uint32_t)gi * 4u : BUF_OOB;
            x = buf_load4(rin, off);
            gm = bt = f4{0.f, 0.f, 0.f, 0.f};
            if (ln) {
                gm = buf_load4(rgm, off);
                bt = buf_load4(rbt, off);
            }
            return sv;
        }
        x = gm = bt = f4{0.f, 0.f, 0.f, 0.f};
        if (!sv) return false;
        {
#pragma unroll
            for (int j = 0; j < 4; j++)
                if (k0 + j < a.K) {
                    x[j] = inb[gi + j];
                    if (ln) {
                        gm[j] = a.gamma[a.in_off + gi + j];
                        bt[j] = a.beta[a.in_off + gi + j];
                    }
                }
        }
        return true;
    };
    if (all_taps) {   // every tap's weights staged once
        for (int tap = 0; tap < a.taps; tap++) stage_w(tap, wsm + (size_t)tap * nw);
    }
    const int total = a.taps * G;
    f4 xn, gn, bn;
    bool vn = load(0, 0, xn, gn, bn);
    // (tap, g) of step it and of step it + 1, advanced incrementally: an integer division per step is
    // ~30 VALU instructions even on uniform operands
    int tap = 0, g = 0, tap1 = G == 1 ? 1 : 0, g1 = G == 1 ? 0 : 1;
    for (int it = 0; it < total; it++) {
        f4 x = xn, gm = gn, bt = bn;
        const bool v = vn;
        if (g == 0 && !all_taps) {
            __syncthreads();   // the previous tap's B reads are done
            stage_w(tap, wsm);
        }
        if (it + 1 < total) vn = load(tap1, g1, xn, gn, bn);
        if (g == 0 && (!all_taps ? true : tap == 0)) __syncthreads();
        if (VEC || v) {   // (VEC: invalid lanes hold zeros, which this maps to 0)
            if (ln) {
#pragma unroll
                for (int j = 0; j < 4; j++) x[j] = (lrelu(x[j]) - mu) * rs * gm[j] + bt[j];
            } else if (a.act) {
#pragma unroll
                for (int j = 0; j < 4; j++) x[j] = lrelu(x[j]);
            }
        }
        const f4* bw = reinterpret_cast<const f4*>(wsm + (all_taps ? (size_t)tap * nw : 0)) + (size_t)(4 * g + kq) * NS + i16;
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const f4 bv = bw[16 * m];
#pragma unroll
            for (int s = 0; s < 4; s++) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[s], bv[s], acc[m], 0, 0, 0);
        }
        tap = tap1;
        g = g1;
        if (++g1 == G) {
            g1 = 0;
            tap1++;
        }
    }
    // acc[m][rr] = out[pixel p0 + 16 wave + 4 kq + rr][channel n0 + 16 m + i16]
    const bool lnr = a.lnr_part != nullptr;
    const float lmu = lnr ? a.lnr_stats[2 * b] : 0.f, lrs = lnr ? a.lnr_stats[2 * b + 1] : 0.f;
    double sg = 0.0, sgh = 0.0;
    // the LN reduction's operands (raw LN input, gamma) of every element, loaded before any store
    float lx[4][NR], lg[4][NR];
    if (lnr) {
#pragma unroll
        for (int rr = 0; rr < 4; rr++) {
            const int p = min(p0 + wave * 16 + 4 * kq + rr, npx - 1);
#pragma unroll
            for (int m = 0; m < NR; m++) {
                const int n = min(n0 + 16 * m + i16, a.N - 1);
                lx[rr][m] = a.lnr_x[((size_t)b * npx + p) * a.out_cs + a.out_off + n];
                lg[rr][m] = a.lnr_gamma[(size_t)p * a.out_cs + a.out_off + n];
            }
        }
    }
#pragma unroll
    for (int rr = 0; rr < 4; rr++) {
        const int p = p0 + wave * 16 + 4 * kq + rr;
        if (p >= npx) continue;
        const size_t ob = ((size_t)b * npx + p) * a.out_cs + a.out_off;
#pragma unroll
        for (int m = 0; m < NR; m++) {
            const int n = n0 + 16 * m + i16;
            if (n >= a.N) continue;
            float v = acc[m][rr];
            if (a.bias) v += a.bias[n];
            if (a.res) v += a.res[ob + n];
            if (a.accumulate) v += a.out[ob + n];
            a.out[ob + n] = v;
            if (lnr) {
                const float g = v * lg[rr][m], xh = (lrelu(lx[rr][m]) - lmu) * lrs;
                sg += g;
                sgh += (double)g * xh;
            }
        }
    }
    if (lnr) lnr_finish(a, sg, sgh, b);
}

// ------------------------------------------------------------------------------------------------
// k_tconv_band: 3x3 (dilation <= 2) convolution, forward or transposed, for images of width <= 64.
// A workgroup owns TH full rows (TH * W <= 64 pixels, 16 per wave) x 16*NR output channels of one
// image. Per 64-channel chunk of K the input band (rows r0 - d .. r0 + TH + d, columns -d .. W + d)
// is staged into LDS once, LN + LeakyReLU applied once per element and zero padding written, so
// the nine taps read their A operands from LDS (one float4 per lane and group) instead of
// re-reading global memory per tap; the chunk's weights for every tap sit in LDS as in
// k_tconv_mfma ([tap][g][kq][j][s]).
// ------------------------------------------------------------------------------------------------
constexpr int TB_KS = 68;   // band pixel stride (floats)

template <int NR, int SUB>
__global__ __launch_bounds__(256) void k_tconv_band(TConvArgs a, int TH, int all_taps) {
    extern __shared__ __attribute__((aligned(16))) float tsm[];
    constexpr int NS = 16 * NR;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i16 = lane & 15, kq = lane >> 4;
    const int H = a.H, W = a.W, npx = H * W, b = blockIdx.y;
    const int r0 = blockIdx.x * TH, n0 = blockIdx.z * NS;
    const int d = a.dil, BW = W + 2 * d, BH = TH + 2 * d;
    float* band = tsm;                                   // [BH * BW][TB_KS]
    float* wl = tsm + (size_t)BH * BW * TB_KS;           // [tap][16 gq][NS][4] of the chunk (all_taps) or one tap
    // the lane's A pixel of subtile s inside the tile: (wave + 4 s) * 16 + i16
    int tr[SUB], tc[SUB];
    bool pav[SUB];
#pragma unroll
    for (int s = 0; s < SUB; s++) {
        const int p = (wave + 4 * s) * 16 + i16;
        tr[s] = p / W;
        tc[s] = p - tr[s] * W;
        pav[s] = p < TH * W && r0 + tr[s] < H;
    }
    const float* inb = a.in + (size_t)b * npx * a.in_cs + a.in_off;
    const bool ln = a.stats != nullptr;
    const float mu = ln ? a.stats[2 * b] : 0.f, rs = ln ? a.stats[2 * b + 1] : 1.f;
    f4 acc[SUB][NR];
#pragma unroll
    for (int s = 0; s < SUB; s++)
#pragma unroll
        for (int m = 0; m < NR; m++) acc[s][m] = f4{0.f, 0.f, 0.f, 0.f};
    const bool vq = (a.in_cs & 3) == 0 && (a.in_off & 3) == 0;
    const uint32_t inbytes = (uint32_t)(npx * a.in_cs - a.in_off) * 4u;
    const __amdgpu_buffer_rsrc_t rin = buf_rsrc(inb, inbytes);
    const __amdgpu_buffer_rsrc_t rgm = buf_rsrc(ln ? a.gamma + a.in_off : inb, inbytes);
    const __amdgpu_buffer_rsrc_t rbt = buf_rsrc(ln ? a.beta + a.in_off : inb, inbytes);
    // whole quads of K from 16-byte loads (and aligned gamma / beta): the branch-free staging path
    const bool fullq = vq && (a.K & 3) == 0 && (!ln || ((((uintptr_t)a.gamma) | ((uintptr_t)a.beta)) & 15) == 0);
    const uint32_t m_bw = udiv_magic(BW);
    for (int kc = 0; kc < a.K; kc += 64) {
        // quads up to the 16-channel group boundary (the MFMA reads whole groups: zeros past K)
        const int KC = min(64, a.K - kc), cq = ((KC + 15) >> 4) * 4;
        __syncthreads();   // the previous chunk's reads are done
        // band: quads of KC channels (zero beyond KC / outside the image), LN on load
        const int nq = BH * BW * cq;
        const uint32_t m_cq = udiv_magic(cq);
        constexpr int TBU = 4;   // band quads per thread and load batch (8 / 16 measured slower)
        for (int e0 = threadIdx.x; e0 < nq; e0 += 256 * TBU) {
            f4 v[TBU];
            int lo[TBU];
#pragma unroll
            for (int u = 0; u < TBU; u++) {
                const int e = e0 + 256 * u;
                v[u] = f4{0.f, 0.f, 0.f, 0.f};
                const int pb = udiv(e, m_cq), q = e - pb * cq;
                lo[u] = pb * TB_KS + 4 * q;
                const int br = udiv(pb, m_bw), bc = pb - br * BW;
                const int r = r0 - d + br, c = bc - d, k = kc + 4 * q;
                const bool in = e < nq && r >= 0 && r < H && c >= 0 && c < W;
                if (fullq) {
                    // branch-free: lanes outside the image (or past K) read zeros for x, gamma and beta,
                    // which the LN / LeakyReLU map to exactly 0
                    const bool ok = in && k < a.K;
                    const uint32_t off = ok ? (uint32_t)((r * W + c) * a.in_cs + k) * 4u : BUF_OOB;
                    const f4 x = buf_load4(rin, off);
                    if (ln) {
                        const f4 gq = buf_load4(rgm, off);
                        const f4 bq = buf_load4(rbt, off);
#pragma unroll
                        for (int jj = 0; jj < 4; jj++) v[u][jj] = (lrelu(x[jj]) - mu) * rs * gq[jj] + bq[jj];
                    } else {
#pragma unroll
                        for (int jj = 0; jj < 4; jj++) v[u][jj] = a.act ? lrelu(x[jj]) : x[jj];
                    }
                } else if (in) {
                    {
                        const size_t gi = ((size_t)r * W + c) * a.in_cs + k;
                        f4 x = f4{0.f, 0.f, 0.f, 0.f}, gm = f4{1.f, 1.f, 1.f, 1.f}, bt = f4{0.f, 0.f, 0.f, 0.f};
                        if (vq && k + 4 <= a.K) {
                            x = *reinterpret_cast<const f4*>(inb + gi);
                            if (ln) {
                                gm = *reinterpret_cast<const f4*>(a.gamma + a.in_off + gi);
                                bt = *reinterpret_cast<const f4*>(a.beta + a.in_off + gi);
                            }
                        } else {
#pragma unroll
                            for (int j = 0; j < 4; j++)
                                if (k + j < a.K) {
                                    x[j] = inb[gi + j];
                                    if (ln) {
                                        gm[j] = a.gamma[a.in_off + gi + j];
                                        bt[j] = a.beta[a.in_off + gi + j];
                                    }
                                }
                        }
#pragma unroll
                        for (int j = 0; j < 4; j++) {
                            const float t = (a.act || ln) ? lrelu(x[j]) : x[j];
                            v[u][j] = k + j < a.K ? (ln ? (t - mu) * rs * gm[j] + bt[j] : t) : 0.f;
                        }
                    }
                }
            }
#pragma unroll
            for (int u = 0; u < TBU; u++)
                if (e0 + 256 * u < nq) *reinterpret_cast<f4*>(band + lo[u]) = v[u];
        }
        // weights of the chunk: [tap][gq = 4g + kq'][j][s], k = kc + 16g + 4kq' + s, gq < GQ = 4 * the
        // chunk's 16-channel groups (every tap at once when they fit next to the band, else one tap at a
        // time; a 2-channel K stages 4 gq rows per tap, not 16)
        const int GQ = 4 * ((KC + 15) >> 4);
        const uint32_t m_gq = udiv_magic(GQ);
        // (buffer loads need 4-byte alignment only: the conv's offset in the dense image may be any float)
        const bool wvec = a.wk == 1 && (a.wn & 3) == 0 && (a.K & 3) == 0 && (kc & 3) == 0 && a.wt * 9 < (1LL << 29);
        const __amdgpu_buffer_rsrc_t rw = buf_rsrc(a.w, (uint32_t)((a.wt * 9) * 4));
        auto stage_w = [&](int t0, int nt) {
            const int nwc = nt * GQ * NS * 4;
            if (wvec) {
                // a data gradient's weights (wk == 1): the 4 k of an s-quad are consecutive in the dense
                // image, one 16-byte buffer load per (tap, gq, j); out-of-range k / n read 0
                const int nw4 = nwc >> 2;
                for (int e0 = threadIdx.x; e0 < nw4; e0 += 256 * TW_U) {
                    f4 v[TW_U];
#pragma unroll
                    for (int u = 0; u < TW_U; u++) {
                        const int e = e0 + 256 * u;
                        const int j = e % NS, rest = e / NS;
                        const int tq = udiv(rest, m_gq), tap = t0 + tq, gq = rest - tq * GQ;
                        const int k = kc + 4 * gq, n = n0 + j;
                        const bool ok = e < nw4 && k < a.K && n < a.N;
                        v[u] = buf_load4(rw, ok ? (uint32_t)(tap * (int)a.wt + n * a.wn + k) * 4u : BUF_OOB);
                    }
#pragma unroll
                    for (int u = 0; u < TW_U; u++)
                        if (e0 + 256 * u < nw4) *reinterpret_cast<f4*>(wl + 4 * (e0 + 256 * u)) = v[u];
                }
                return;
            }
            for (int e0 = threadIdx.x; e0 < nwc; e0 += 256 * TW_U) {
                float v[TW_U];
#pragma unroll
                for (int u = 0; u < TW_U; u++) {
                    const int e = e0 + 256 * u;
                    const int s4 = e & 3, j = (e >> 2) % NS, rest = (e >> 2) / NS;   // rest = tap' * GQ + gq
                    const int tq = udiv(rest, m_gq), tap = t0 + tq, gq = rest - tq * GQ;
                    const int k = kc + 4 * gq + s4, n = n0 + j;
                    const bool ok = e < nwc && k < a.K && n < a.N;
                    v[u] = *(ok ? a.w + (tap * a.wt + (long long)k * a.wk + (long long)n * a.wn) : a.zero);
                }
#pragma unroll
                for (int u = 0; u < TW_U; u++)
                    if (e0 + 256 * u < nwc) wl[e0 + 256 * u] = v[u];
            }
        };
        if (all_taps) stage_w(0, 9);
        __syncthreads();
        const int G = (KC + 15) >> 4;
#pragma unroll 1
        for (int tap = 0; tap < 9; tap++) {
            if (!all_taps) {
                if (tap > 0) __syncthreads();   // the previous tap's weight reads are done
                stage_w(tap, 1);
                __syncthreads();
            }
            const int dr = tap / 3 - 1, dc = tap % 3 - 1;
            const f4* wp = reinterpret_cast<const f4*>(wl) + (size_t)(all_taps ? tap : 0) * GQ * NS + (size_t)kq * NS + i16;
            const float* ap[SUB];
#pragma unroll
            for (int s = 0; s < SUB; s++) {
                const int br = tr[s] + d + a.sgn * d * dr, bc = tc[s] + d + a.sgn * d * dc;
                ap[s] = band + (size_t)(br * BW + bc) * TB_KS + 4 * kq;
            }
            for (int g = 0; g < G; g++) {
                f4 x[SUB];
#pragma unroll
                for (int s = 0; s < SUB; s++) x[s] = pav[s] ? *reinterpret_cast<const f4*>(ap[s] + 16 * g) : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int m = 0; m < NR; m++) {
                    const f4 bv = wp[(size_t)4 * g * NS + 16 * m];
#pragma unroll
                    for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
                        for (int s = 0; s < SUB; s++)
                            acc[s][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[s][s4], bv[s4], acc[s][m], 0, 0, 0);
                }
            }
        }
    }
    // acc[s][m][rr] = out[tile pixel (wave + 4s) * 16 + 4 kq + rr][channel n0 + 16 m + i16]
    const bool lnr = a.lnr_part != nullptr;
    const float lmu = lnr ? a.lnr_stats[2 * b] : 0.f, lrs = lnr ? a.lnr_stats[2 * b + 1] : 0.f;
    double sg = 0.0, sgh = 0.0;
    // the LN reduction's operands (raw LN input, gamma) of every element, loaded before any store
    float lx[SUB][4][NR], lg[SUB][4][NR];
    if (lnr) {
#pragma unroll
        for (int s = 0; s < SUB; s++)
#pragma unroll
            for (int rr = 0; rr < 4; rr++) {
                const int q = (wave + 4 * s) * 16 + 4 * kq + rr;
                const int orow = min(r0 + q / W, H - 1), ocol = q % W;
                const size_t pix = (size_t)orow * W + ocol;
#pragma unroll
                for (int m = 0; m < NR; m++) {
                    const int n = min(n0 + 16 * m + i16, a.N - 1);
                    lx[s][rr][m] = a.lnr_x[((size_t)b * npx + pix) * a.out_cs + a.out_off + n];
                    lg[s][rr][m] = a.lnr_gamma[pix * a.out_cs + a.out_off + n];
                }
            }
    }
#pragma unroll
    for (int s = 0; s < SUB; s++)
#pragma unroll
        for (int rr = 0; rr < 4; rr++) {
            const int q = (wave + 4 * s) * 16 + 4 * kq + rr;
            const int orow = r0 + q / W, ocol = q % W;
            if (q >= TH * W || orow >= H) continue;
            const size_t pix = (size_t)orow * W + ocol;
            const size_t ob = ((size_t)b * npx + pix) * a.out_cs + a.out_off;
#pragma unroll
            for (int m = 0; m < NR; m++) {
                const int n = n0 + 16 * m + i16;
                if (n >= a.N) continue;
                float v = acc[s][m][rr];
                if (a.bias) v += a.bias[n];
                if (a.res) v += a.res[ob + n];
                if (a.accumulate) v += a.out[ob + n];
                a.out[ob + n] = v;
                if (lnr) {
                    const float g = v * lg[s][rr][m], xh = (lrelu(lx[s][rr][m]) - lmu) * lrs;
                    sg += g;
                    sgh += (double)g * xh;
                }
            }
        }
    if (lnr) lnr_finish(a, sg, sgh, b);
}

// ------------------------------------------------------------------------------------------------
// k_tconv_thin: a 3x3 (dilation 1) convolution with K <= 4 input channels, forward or transposed, no
// LN on load: the streamed conv_out's data gradient (K = dc2 -> N = nk, with the fused LN_out
// reduction) and conv_in's forward recompute (K = dc1). The MFMA kernels pad such a K to a 16-wide
// group and stage per-tap weights for 2 useful channels; here a workgroup owns TR full rows
// (TR * W <= 64 pixels at N = 64) of one image, stages the K-channel band (1-pixel halo, zeros
// outside) and the 9 * K * N weights in LDS; each thread computes up to 4 pixels x 4 channels on the
// vector ALUs (tap outer: one weight quad read per tap and k), then issues every epilogue load (residual / previous
// output / the LN reduction's raw input and gamma) before its float4 stores.
// ------------------------------------------------------------------------------------------------
template <int K>
__global__ __launch_bounds__(256, 2) void k_tconv_thin(TConvArgs a, int TR) {
    extern __shared__ __attribute__((aligned(16))) float tsm[];
    constexpr int PX = 4;   // pixels per thread (TR * W <= 4 * 256 / (N / 4))
    const int H = a.H, W = a.W, npx = H * W, b = blockIdx.y, N = a.N;
    const int r0 = blockIdx.x * TR, BW = W + 2, BH = TR + 2;
    const int nb = (BH * BW * K + 3) & ~3;
    float* ws = tsm + nb;   // [tap][k][N] weights
    const float* inb = a.in + (size_t)b * npx * a.in_cs + a.in_off;
    for (int e = threadIdx.x; e < BH * BW * K; e += 256) {
        const int pb = e / K, k = e - pb * K;
        const int br = pb / BW, bc = pb - br * BW;
        const int r = r0 - 1 + br, c = bc - 1;
        float v = 0.f;
        if (r >= 0 && r < H && c >= 0 && c < W) {
            v = inb[(size_t)(r * W + c) * a.in_cs + k];
            if (a.act) v = lrelu(v);
        }
        tsm[e] = v;
    }
    for (int e = threadIdx.x; e < 9 * K * N; e += 256) {
        const int tk = e / N, n = e - tk * N, tap = tk / K, k = tk - tap * K;
        ws[e] = a.w[tap * a.wt + (long long)k * a.wk + (long long)n * a.wn];
    }
    const int NQ = N >> 2, PS = 256 / NQ;
    const int qd = threadIdx.x % NQ, ps = threadIdx.x / NQ, n0 = 4 * qd;
    f4 bias = f4{0.f, 0.f, 0.f, 0.f};
    if (a.bias)
#pragma unroll
        for (int j = 0; j < 4; j++) bias[j] = a.bias[n0 + j];
    const int ntp = min(TR, H - r0) * W;   // this tile's pixels
    int xo[PX], ob[PX];   // band float offset of the pixel (tap (1, 1)); output float offset
    f4 acc[PX];
#pragma unroll
    for (int i = 0; i < PX; i++) {
        const int px = min(ps + PS * i, ntp - 1);
        const int pr = px / W, pc = px - pr * W;
        xo[i] = ((pr + 1) * BW + pc + 1) * K;
        ob[i] = ((b * npx + (r0 + pr) * W + pc) * a.out_cs + a.out_off + n0);
        acc[i] = bias;
    }
    __syncthreads();
    // tap outer, pixels inner: each weight quad is read from LDS once per thread
#pragma unroll
    for (int tap = 0; tap < 9; tap++) {
        const int dr = tap / 3 - 1, dc = tap % 3 - 1;
        const int toff = (a.sgn * dr * BW + a.sgn * dc) * K;
#pragma unroll
        for (int k = 0; k < K; k++) {
            const f4 wq = *reinterpret_cast<const f4*>(ws + (tap * K + k) * N + n0);
#pragma unroll
            for (int i = 0; i < PX; i++) {
                const float x = tsm[xo[i] + toff + k];
#pragma unroll
                for (int j = 0; j < 4; j++) acc[i][j] = fmaf(x, wq[j], acc[i][j]);
            }
        }
        __builtin_amdgcn_sched_barrier(0);   // one tap's LDS reads live at a time (else all 9 are hoisted)
    }
    const bool lnr = a.lnr_part != nullptr;
    // (gamma lives in the parameter vector at any float offset: a 16-byte buffer load needs 4-byte
    // alignment only)
    const __amdgpu_buffer_rsrc_t rlg = buf_rsrc(lnr ? a.lnr_gamma : a.out, (uint32_t)(npx * a.out_cs) * 4u);
    // (out-of-tile slots were clamped to the tile's last pixel above: every load is in range, only the
    // stores and the sums are predicated — no control flow around the per-pixel arrays)
    f4 lx[PX], lg[PX];
#pragma unroll
    for (int i = 0; i < PX; i++) {
        if (a.res) acc[i] += *reinterpret_cast<const f4*>(a.res + ob[i]);
        if (a.accumulate) acc[i] += *reinterpret_cast<const f4*>(a.out + ob[i]);
        if (lnr) {
            lx[i] = *reinterpret_cast<const f4*>(a.lnr_x + ob[i]);
            lg[i] = buf_load4(rlg, (uint32_t)(ob[i] - b * npx * a.out_cs) * 4u);
        }
    }
    const float lmu = lnr ? a.lnr_stats[2 * b] : 0.f, lrs = lnr ? a.lnr_stats[2 * b + 1] : 0.f;
    double sg = 0.0, sgh = 0.0;
#pragma unroll
    for (int i = 0; i < PX; i++) {
        const bool ok = ps + PS * i < ntp;
        const f4 v = acc[i];
        if (ok) *reinterpret_cast<f4*>(a.out + ob[i]) = v;
        if (lnr)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float g = ok ? v[j] * lg[i][j] : 0.f, xh = (lrelu(lx[i][j]) - lmu) * lrs;
                sg += g;
                sgh += (double)g * xh;
            }
    }
    if (lnr) lnr_finish(a, sg, sgh, b);
}

// debug option TRAIN_ALT bit 8: no thin-K convolutions (the MFMA kernels take them)
static bool tconv_thin_on() { return (opts().train_alt & 8) == 0; }

// debug option TRAIN_ALT bit 1: the register-blocked VALU kernels
static bool train_valu() { return (opts().train_alt & 1) != 0; }
bool train_valu_kernels() { return train_valu(); }

int launch_tconv(const TConvArgs& a_in, hipStream_t st) {
    TConvArgs a = a_in;
    const int npx = a.H * a.W;
    // a fused LN reduction writes one partial per workgroup of an image: drop it where there are too many
    auto lnr_ok = [&](const dim3& g) {
        if (a.lnr_part != nullptr && a.lnr_base + (int)(g.x * g.z) > a.lnr_stride) a.lnr_part = nullptr;
        return a.lnr_part != nullptr ? (int)(g.x * g.z) : 0;
    };
    const bool band_off = (opts().train_alt & 4) != 0;   // debug option TRAIN_ALT bit 4: no band-staged 3x3 kernel
    auto al16 = [](const void* p) { return ((uintptr_t)p & 15) == 0; };
    if (!train_valu() && tconv_thin_on() && a.taps == 9 && a.dil == 1 && a.K >= 1 && a.K <= 4 &&
        a.stats == nullptr && (a.N == 64 || a.N == 32 || a.N == 16) && a.W >= 1 && (a.out_cs & 3) == 0 &&
        (a.out_off & 3) == 0 && al16(a.out) && (a.res == nullptr || al16(a.res)) &&
        (a.lnr_part == nullptr || al16(a.lnr_x)) && (long long)a.B * a.H * a.W * a.out_cs < (1LL << 31)) {
        const int PS = 256 / (a.N / 4);
        const int TR = std::max(1, std::min(a.H, PS * 4 / a.W));
        if (TR * a.W <= PS * 4) {
            const dim3 g((a.H + TR - 1) / TR, a.B, 1), blk(256);
            const int np = lnr_ok(g);
            const size_t lds = (((size_t)(TR + 2) * (a.W + 2) * a.K + 3) / 4 * 4 + (size_t)9 * a.K * a.N) * 4;
            switch (a.K) {
                case 1: hipLaunchKernelGGL((k_tconv_thin<1>), g, blk, lds, st, a, TR); break;
                case 2: hipLaunchKernelGGL((k_tconv_thin<2>), g, blk, lds, st, a, TR); break;
                case 3: hipLaunchKernelGGL((k_tconv_thin<3>), g, blk, lds, st, a, TR); break;
                default: hipLaunchKernelGGL((k_tconv_thin<4>), g, blk, lds, st, a, TR); break;
            }
            return np;
        }
    }
    if (!train_valu() && !band_off && a.taps == 9 && a.dil <= 2 && a.W <= 64 && a.W >= 1) {
        const int nr = a.N <= 16 ? 1 : a.N <= 32 ? 2 : a.N <= 48 ? 3 : 4;
        const int NS = 16 * nr;
        // one tap of a chunk's weights: 4 gq rows per 16-channel group of the (at most 64) chunk channels
        const size_t w1 = (size_t)4 * ((std::min(64, a.K) + 15) / 16) * NS * 4 * 4;
        // subtiles per wave: tiles of 64 * SUB pixels amortise the weight staging and the halo rows over
        // more outputs, while the launch keeps >= 512 workgroups (two per CU) and the band fits LDS
        int sub = 1;
        for (int s : {4, 2}) {
            if (sub > 1 || s * nr > 4) continue;   // (acc registers: SUB * NR <= 4)
            const int TH = std::max(1, std::min(a.H, 64 * s / a.W));
            const long long wgs = (long long)((a.H + TH - 1) / TH) * a.B * ((a.N + NS - 1) / NS);
            const size_t band = (size_t)(TH + 2 * a.dil) * (a.W + 2 * a.dil) * TB_KS * 4;
            // (measured at cfg2 B=64, train step, same box: minimum 1024 workgroups 12.17 ms, 512 12.10,
            // 256 11.79 -- the 32x32 branch dgrads then run SUB=4, 256 workgroups of 8 rows, a quarter of
            // the per-workgroup weight staging and halo rows)
            constexpr long long minwg = 256;
            if (64 * s <= a.H * a.W && wgs >= minwg && band + w1 <= 160 * 1024) sub = s;
        }
        const int TH = std::max(1, std::min(a.H, 64 * sub / a.W));
        const size_t band = (size_t)(TH + 2 * a.dil) * (a.W + 2 * a.dil) * TB_KS * 4;
        // LDS budget (KiB) for staging every tap's weights at once
        const long long at_lim = sub > 1 ? 156 : 80;
        const int all_taps = (long long)(band + 9 * w1) <= at_lim * 1024 ? 1 : 0;
        const size_t lds = band + (all_taps ? 9 : 1) * w1;
        if (lds <= 160 * 1024) {
            const dim3 g((a.H + TH - 1) / TH, a.B, (a.N + NS - 1) / NS), blk(256);
            const int np = lnr_ok(g);
            if (sub == 4)
                hipLaunchKernelGGL((k_tconv_band<1, 4>), g, blk, lds, st, a, TH, all_taps);
            else if (sub == 2 && nr == 1)
                hipLaunchKernelGGL((k_tconv_band<1, 2>), g, blk, lds, st, a, TH, all_taps);
            else if (sub == 2)
                hipLaunchKernelGGL((k_tconv_band<2, 2>), g, blk, lds, st, a, TH, all_taps);
            else if (nr == 1)
                hipLaunchKernelGGL((k_tconv_band<1, 1>), g, blk, lds, st, a, TH, all_taps);
            else if (nr == 2)
                hipLaunchKernelGGL((k_tconv_band<2, 1>), g, blk, lds, st, a, TH, all_taps);
            else if (nr == 3)
                hipLaunchKernelGGL((k_tconv_band<3, 1>), g, blk, lds, st, a, TH, all_taps);
            else
                hipLaunchKernelGGL((k_tconv_band<4, 1>), g, blk, lds, st, a, TH, all_taps);
            return np;
        }
    }
    if (!train_valu()) {
        const int nr = a.N <= 16 ? 1 : a.N <= 32 ? 2 : a.N <= 48 ? 3 : 4;
        const int NS = 16 * nr;
        const int G = (a.K + 15) / 16;
        const size_t lds1 = (size_t)G * 16 * NS * 4;
        if (lds1 <= 64 * 1024) {
            // every tap's weights in LDS at once when they fit (no per-tap barriers), else per tap
            const int all_taps = lds1 * a.taps <= 64 * 1024 ? 1 : 0;
            const size_t lds = all_taps ? lds1 * a.taps : lds1;
            const bool vec = a.K % 4 == 0 && a.in_cs % 4 == 0 && a.in_off % 4 == 0;
            const dim3 g((npx + 63) / 64, a.B, (a.N + NS - 1) / NS), blk(256);
            const int np = lnr_ok(g);
#define CNF_TM(NR_)                                                                                   \
    if (nr == NR_) {                                                                                  \
        if (vec)                                                                                      \
            hipLaunchKernelGGL((k_tconv_mfma<NR_, true>), g, blk, lds, st, a, all_taps);            \
        else                                                                                          \
            hipLaunchKernelGGL((k_tconv_mfma<NR_, false>), g, blk, lds, st, a, all_taps);           \
        return np;                                                                                    \
    }
            CNF_TM(1) CNF_TM(2) CNF_TM(3) CNF_TM(4)
#undef CNF_TM
        }
    }
    const int TN = a.N <= 4 ? 4 : a.N <= 16 ? 16 : 64;
    const int TP = 4096 / TN;
    const dim3 g((npx + TP - 1) / TP, a.B, (a.N + TN - 1) / TN), blk(256);
    if (TN == 4)
        hipLaunchKernelGGL(k_tconv<4>, g, blk, 0, st, a);
    else if (TN == 16)
        hipLaunchKernelGGL(k_tconv<16>, g, blk, 0, st, a);
    else
        hipLaunchKernelGGL(k_tconv<64>, g, blk, 0, st, a);
    return 0;   // (the VALU kernel has no fused LN reduction)
}

// ------------------------------------------------------------------------------------------------
// k_wgrad: grid (chunks, taps, ci-blocks x co-blocks); a chunk is a run of chunk_px pixels of the
// flattened (image, pixel) axis, consumed 16 pixels per step through LDS.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_wgrad(WGradArgs a) {
    constexpr int SP = 16, XS = 68;
    __shared__ __attribute__((aligned(16))) float Xs[SP * XS];
    __shared__ __attribute__((aligned(16))) float Ds[SP * XS];
    const int t = threadIdx.x, tx = t & 15, ty = t >> 4;
    const int npx = a.H * a.W;
    const long long total = (long long)a.B * npx;
    const int tap = blockIdx.y;
    const int nco = (a.CO + 63) / 64;
    const int ci0 = (blockIdx.z / nco) * 64, co0 = (blockIdx.z % nco) * 64;
    const int dr = a.taps == 1 ? 0 : tap / 3 - 1, dc = a.taps == 1 ? 0 : tap % 3 - 1;
    const long long g0 = (long long)blockIdx.x * a.chunk_px;
    const long long g1 = g0 + a.chunk_px < total ? g0 + a.chunk_px : total;
    const bool do_bias = a.bpart != nullptr && tap == 0 && ci0 == 0;
    float acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < 4; j++) acc[i][j] = 0.f;
    float bacc[4] = {0.f, 0.f, 0.f, 0.f};
    for (long long gs = g0; gs < g1; gs += SP) {
        for (int e = t; e < SP * 64; e += 256) {
            const int c = e & 63, px = e >> 6;
            const long long g = gs + px;
            float xv = 0.f, dv = 0.f;
            if (g < g1) {
                const int b = (int)(g / npx), p = (int)(g - (long long)b * npx);
                if (co0 + c < a.CO) dv = a.dy[((size_t)b * npx + p) * a.dy_cs + a.dy_off + co0 + c];
                if (ci0 + c < a.CI) {
                    const int r = p / a.W + a.dil * dr, cc = p % a.W + a.dil * dc;
                    if (r >= 0 && r < a.H && cc >= 0 && cc < a.W) {
                        const size_t q = (size_t)r * a.W + cc;
                        const size_t gi = q * a.x_cs + a.x_off + ci0 + c;
                        xv = act_load(a.x[(size_t)b * npx * a.x_cs + gi], a.act, a.stats, a.gamma, a.beta, b, gi);
                    }
                }
            }
            Xs[px * XS + c] = xv;
            Ds[px * XS + c] = dv;
        }
        __syncthreads();
#pragma unroll
        for (int px = 0; px < SP; px++) {
            const f4 x = *reinterpret_cast<const f4*>(&Xs[px * XS + 4 * tx]);
            const f4 d = *reinterpret_cast<const f4*>(&Ds[px * XS + 4 * ty]);
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 4; j++) acc[i][j] = fmaf(x[i], d[j], acc[i][j]);
            if (do_bias && tx == 0) {
#pragma unroll
                for (int j = 0; j < 4; j++) bacc[j] += d[j];
            }
        }
        __syncthreads();
    }
    float* part = a.part + (size_t)blockIdx.x * a.taps * a.CI * a.CO;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const int ci = ci0 + 4 * tx + i;
        if (ci >= a.CI) continue;
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int co = co0 + 4 * ty + j;
            if (co < a.CO) part[((size_t)tap * a.CI + ci) * a.CO + co] = acc[i][j];
        }
    }
    if (do_bias && tx == 0) {
#pragma unroll
        for (int j = 0; j < 4; j++) {
            const int co = co0 + 4 * ty + j;
            if (co < a.CO) a.bpart[(size_t)blockIdx.x * a.CO + co] = bacc[j];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// k_wgrad_band: weight gradient of a 3x3 (TR = 3) or 1x1 (TR = 1) conv on MFMA with every tap of
// one kernel row per workgroup. Work units are (image, band of RB rows); a workgroup of grid
// column `chunk` takes units chunk, chunk + chunks, ... For each unit it stages the X rows its
// tap row reads (dilation halo columns, zero padding, LN + LeakyReLU applied once per element)
// and the dY rows into LDS, then runs K = the unit's pixels through the MFMAs: the B operand
// (dY) is read once per k-step and shared by the TR taps. Wave w owns ci rows 16w.. of the
// 64 x 64 (ci, co) tile: acc[t][m][r] = dW[tap row, t][ci 16w+4kq+r][co 16m+i16]. The bias
// gradient (sum of dY) goes after the weights in the same partial row, so one scatter launch
// reduces both.
// ------------------------------------------------------------------------------------------------
__host__ __device__ constexpr int wg_stride(int c) {   // LDS row stride == 16 (mod 32) floats
    return ((c + 15) / 16 * 16) % 32 == 0 ? (c + 15) / 16 * 16 + 16 : (c + 15) / 16 * 16;
}

// (at least 3 waves per SIMD: the launch fits 2-3 workgroups per CU by LDS, and without the bound the
// 8-deep staging loads took 266 registers, one wave per SIMD)
constexpr int WG_U = 4;   // staging loads in flight per thread and array
template <int TR>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3))) void k_wgrad_band(WGradArgs a, int RB,
                                                                                          int nunits) {
    extern __shared__ __attribute__((aligned(16))) float wsm[];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, i16 = lane & 15, kq = lane >> 4;
    const int H = a.H, W = a.W, npx = H * W;
    const int nco = (a.CO + 63) / 64;
    const int ci0 = (blockIdx.z / nco) * 64, co0 = (blockIdx.z % nco) * 64;
    const int CIB = min(64, a.CI - ci0), COB = min(64, a.CO - co0);
    const int XS = wg_stride(CIB), DS = wg_stride(COB);
    const int MB = (COB + 15) >> 4;   // 16-column blocks holding outputs
    // waves -> (ci block, k slice): NCW ci blocks of 16 rows; the waves left over split the k-steps
    // (pixel quads) of every unit and their partial sums are added at the end in a fixed order
    const int NCW = (CIB + 15) >> 4, WPG = NCW == 1 ? 4 : NCW == 2 ? 2 : 1;
    const int cw = wave % NCW, ks = wave / NCW;
    const bool kact = ks < WPG;
    const int hx = TR == 3 ? a.dil : 0;     // halo columns
    const int WB = W + 2 * hx;
    const int dr = TR == 3 ? (int)blockIdx.y - 1 : 0;
    float* Xs = wsm;                          // [RB][WB][XS]
    float* Ds = wsm + (size_t)RB * WB * XS;   // [RB][W][DS]
    const bool do_bias = a.bpart != nullptr && blockIdx.y == (TR == 3 ? 1u : 0u) && ci0 == 0;
    f4 acc[TR][4];
#pragma unroll
    for (int u = 0; u < TR; u++)
#pragma unroll
        for (int m = 0; m < 4; m++) acc[u][m] = f4{0.f, 0.f, 0.f, 0.f};
    float bacc = 0.f;
    const int bands = (H + RB - 1) / RB;
    const bool ln = a.stats != nullptr;
    // quad loads of X need the window quad aligned, and (with LN) 16-byte aligned gamma / beta: they are
    // canonical-parameter pointers (P + offset) with no alignment guarantee of their own
    const bool qx = (CIB & 3) == 0 && (a.x_cs & 3) == 0 && ((a.x_off + ci0) & 3) == 0 &&
                    (!ln || ((((uintptr_t)a.gamma) | ((uintptr_t)a.beta)) & 15) == 0);
    const bool qd = (COB & 3) == 0 && (a.dy_cs & 3) == 0 && ((a.dy_off + co0) & 3) == 0;
    const uint32_t m_cq = udiv_magic(CIB >> 2), m_ci = udiv_magic(CIB), m_wb = udiv_magic(WB), m_dq = udiv_magic(COB >> 2),
                   m_co = udiv_magic(COB);
    for (int unit = blockIdx.x; unit < nunits; unit += gridDim.x) {
        const int b = unit / bands, r0 = (unit - b * bands) * RB;
        const float mu = ln ? a.stats[2 * b] : 0.f, rs = ln ? a.stats[2 * b + 1] : 1.f;
        __syncthreads();   // the previous unit's LDS reads are done
        // X rows r0 + dil*dr .. (+RB), columns -hx .. W + hx; dY rows r0 .. r0 + RB. Channel quads
        // (float4 loads, 8 quads in flight per thread) when the windows are quad aligned.
        const float* xb = a.x + (size_t)b * npx * a.x_cs + a.x_off + ci0;
        const float* db = a.dy + (size_t)b * npx * a.dy_cs + a.dy_off + co0;
        if (qx) {
            const int cq = CIB >> 2, nxq = RB * WB * cq;
            for (int e0 = t; e0 < nxq; e0 += 256 * WG_U) {
                f4 v[WG_U];
                int lo[WG_U];
#pragma unroll
                for (int u = 0; u < WG_U; u++) {
                    const int e = e0 + 256 * u;
                    v[u] = f4{0.f, 0.f, 0.f, 0.f};
                    const int pb = udiv(e, m_cq), c = (e - pb * cq) * 4;
                    lo[u] = pb * XS + c;
                    if (e < nxq) {
                        const int br = udiv(pb, m_wb), bc = pb - br * WB;
                        const int r = r0 + a.dil * dr + br, cc = bc - hx;
                        if (r >= 0 && r < H && cc >= 0 && cc < W) {
                            const size_t gi = ((size_t)r * W + cc) * a.x_cs + c;
                            const f4 xv = *reinterpret_cast<const f4*>(xb + gi);
                            if (ln) {
                                const size_t gg = gi + a.x_off + ci0;
                                const f4 gmv = *reinterpret_cast<const f4*>(a.gamma + gg);
                                const f4 btv = *reinterpret_cast<const f4*>(a.beta + gg);
#pragma unroll
                                for (int j = 0; j < 4; j++) v[u][j] = (lrelu(xv[j]) - mu) * rs * gmv[j] + btv[j];
                            } else {
#pragma unroll
                                for (int j = 0; j < 4; j++) v[u][j] = a.act ? lrelu(xv[j]) : xv[j];
                            }
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < WG_U; u++)
                    if (e0 + 256 * u < nxq) *reinterpret_cast<f4*>(Xs + lo[u]) = v[u];
            }
        } else {
            const int nx = RB * WB * CIB;
            for (int e0 = t; e0 < nx; e0 += 256 * WG_U) {
                float v[WG_U];
                int lo[WG_U];
#pragma unroll
                for (int u = 0; u < WG_U; u++) {
                    const int e = e0 + 256 * u;
                    v[u] = 0.f;
                    const int pb = udiv(e, m_ci), c = e - pb * CIB;
                    lo[u] = pb * XS + c;
                    if (e < nx) {
                        const int br = udiv(pb, m_wb), bc = pb - br * WB;
                        const int r = r0 + a.dil * dr + br, cc = bc - hx;
                        if (r >= 0 && r < H && cc >= 0 && cc < W) {
                            const size_t gi = ((size_t)r * W + cc) * a.x_cs + c;
                            const float xv = xb[gi];
                            if (ln) {
                                const size_t gg = gi + a.x_off + ci0;
                                v[u] = (lrelu(xv) - mu) * rs * a.gamma[gg] + a.beta[gg];
                            } else {
                                v[u] = a.act ? lrelu(xv) : xv;
                            }
                        }
                    }
                }
#pragma unroll
                for (int u = 0; u < WG_U; u++)
                    if (e0 + 256 * u < nx) Xs[lo[u]] = v[u];
            }
        }
        if (qd) {
            const int cq = COB >> 2, ndq = RB * W * cq;
            for (int e0 = t; e0 < ndq; e0 += 256 * WG_U) {
                f4 v[WG_U];
                int lo[WG_U];
#pragma unroll
                for (int u = 0; u < WG_U; u++) {
                    const int e = e0 + 256 * u;
                    v[u] = f4{0.f, 0.f, 0.f, 0.f};
                    const int p = udiv(e, m_dq), c = (e - p * cq) * 4;
                    lo[u] = p * DS + c;
                    if (e < ndq && r0 * W + p < npx)
                        v[u] = *reinterpret_cast<const f4*>(db + ((size_t)r0 * W + p) * a.dy_cs + c);
                }
#pragma unroll
                for (int u = 0; u < WG_U; u++)
                    if (e0 + 256 * u < ndq) *reinterpret_cast<f4*>(Ds + lo[u]) = v[u];
            }
        } else {
            const int nd = RB * W * COB;
            for (int e0 = t; e0 < nd; e0 += 256 * WG_U) {
                float v[WG_U];
                int lo[WG_U];
#pragma unroll
                for (int u = 0; u < WG_U; u++) {
                    const int e = e0 + 256 * u;
                    v[u] = 0.f;
                    const int p = udiv(e, m_co), c = e - p * COB;
                    lo[u] = p * DS + c;
                    if (e < nd && r0 * W + p < npx) v[u] = db[((size_t)r0 * W + p) * a.dy_cs + c];
                }
#pragma unroll
                for (int u = 0; u < WG_U; u++)
                    if (e0 + 256 * u < nd) Ds[lo[u]] = v[u];
            }
        }
        {   // zero the dY rows past the unit's last pixel up to the next multiple of 4
            const int nk = RB * W, nk4 = (nk + 3) & ~3;
            for (int e = t; e < (nk4 - nk) * DS; e += 256) Ds[(size_t)nk * DS + e] = 0.f;
        }
        __syncthreads();
        // K = the unit's pixels, 4 per k-step: lane (i16, kq) reads pixel p = s + kq of the unit, row
        // pr = p / W from a float reciprocal (the 1x1 band has no halo: its pixel is p); past the unit's
        // last pixel dY is zero (padded rows) and X pixel 0 (finite)
        if (kact) {   // column blocks past the outputs have nothing to compute
            const int nk = RB * W, nk4 = (nk + 3) & ~3;
            const float invW = 1.f / (float)W;
            const float* xl = Xs + 16 * cw + i16;
            const float* dl = Ds + (size_t)kq * DS + i16;
            for (int s = 4 * ks; s < nk4; s += 4 * WPG) {
                const int p = s + kq;
                const int pb = TR == 1 ? p : p + (int)(((float)p + 0.5f) * invW) * 2 * hx;   // band pixel
                const int xo = p < nk ? pb * XS : 0;
                float bv[4];
#pragma unroll
                for (int m = 0; m < 4; m++) bv[m] = m < MB ? dl[s * DS + 16 * m] : 0.f;
#pragma unroll
                for (int u = 0; u < TR; u++) {
                    const float av = xl[xo + u * hx * XS];
#pragma unroll
                    for (int m = 0; m < 4; m++)
                        if (m < MB) acc[u][m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[m], acc[u][m], 0, 0, 0);
                }
            }
        }
        if (do_bias && (t & 63) < COB) {   // 4 interleaved pixel slices per column
            const int nk = RB * W;
            for (int p = t >> 6; p < nk; p += 4) bacc += Ds[p * DS + (t & 63)];
        }
    }
    if (do_bias) {   // fixed-order sum of the 4 slices (deterministic)
        __syncthreads();
        Ds[t] = bacc;
        __syncthreads();
        if (t < 64) bacc = Ds[t] + Ds[t + 64] + Ds[t + 128] + Ds[t + 192];
    }
    if (WPG > 1) {   // k slices of one ci block: slice 0 adds the others' sums, in slice order
        float* red = wsm;   // [ks][cw][TR * 16][64 lanes]
        __syncthreads();
        if (ks > 0 && kact) {
#pragma unroll
            for (int u = 0; u < TR; u++)
#pragma unroll
                for (int m = 0; m < 4; m++)
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        red[((size_t)(wave * TR + u) * 16 + m * 4 + r) * 64 + lane] = acc[u][m][r];
        }
        __syncthreads();
        if (ks == 0) {
            for (int k2 = 1; k2 < WPG; k2++) {
                const int w2 = k2 * NCW + cw;
#pragma unroll
                for (int u = 0; u < TR; u++)
#pragma unroll
                    for (int m = 0; m < 4; m++)
#pragma unroll
                        for (int r = 0; r < 4; r++) acc[u][m][r] += red[((size_t)(w2 * TR + u) * 16 + m * 4 + r) * 64 + lane];
            }
        }
    }
    // partial row of this chunk: [taps][CI][CO] weights, then [CO] bias
    float* part = a.part + (size_t)blockIdx.x * ((size_t)a.taps * a.CI * a.CO + a.CO);
#pragma unroll
    for (int u = 0; u < TR; u++) {
        const int tap = TR == 3 ? (int)blockIdx.y * 3 + u : 0;
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int ci = ci0 + 16 * cw + 4 * kq + r;
            if (ks != 0 || ci >= ci0 + CIB) continue;
#pragma unroll
            for (int m = 0; m < 4; m++) {
                const int co = co0 + 16 * m + i16;
                if (co < a.CO) part[((size_t)tap * a.CI + ci) * a.CO + co] = acc[u][m][r];
            }
        }
    }
    if (do_bias && t < COB) part[(size_t)a.taps * a.CI * a.CO + co0 + t] = bacc;
}

// ------------------------------------------------------------------------------------------------
// k_wgrad_direct: weight (and bias) gradient of a 1x1 (TR = 1) or 3x3 (TR = 3) conv on MFMA with both
// operands loaded straight from global memory into registers (no LDS staging, no barriers in the
// loop). The GEMM is dW[r][n] = sum over pixels of A(p, r) G(p, n), r = tap * CI + ci the kernel row
// (A = LN(LeakyReLU(x)) at the tap's shifted pixel, zero outside the image), n < CO. A workgroup owns
// one (image, band of RB rows) unit — its partial row is the unit's — and MT x NT 16x16 blocks of
// (r, n) (grid.y / grid.z tile the rest); its 4 waves take alternate 4-pixel steps along the band's
// rows (width % 4 == 0), each step's loads issued one step ahead of its MFMAs, and their sums are
// added in wave order through LDS (deterministic). The bias gradient (sum of G) is summed on the VALU
// from the same G loads by the grid.y == 0 workgroups. Partial rows as k_wgrad_band: [taps][CI][CO]
// then [CO], reduced by k_grad_scatter.
// ------------------------------------------------------------------------------------------------
template <int MT, int NT, int TR>
__global__ __launch_bounds__(256) void k_wgrad_direct(WGradArgs a, int RB, int nbands) {
    extern __shared__ __attribute__((aligned(16))) float wdsm[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, i16 = lane & 15, kq = lane >> 4;
    const int H = a.H, W = a.W, npx = H * W, CI = a.CI, CO = a.CO;
    const int chunk = blockIdx.x, b = chunk / nbands, y0 = (chunk - b * nbands) * RB, y1 = min(H, y0 + RB);
    const int rows = a.taps * CI, r0 = blockIdx.y * MT * 16, n0 = blockIdx.z * NT * 16;
    const bool ln = a.stats != nullptr, act = ln || a.act;
    const float mu = ln ? a.stats[2 * b] : 0.f, rs = ln ? a.stats[2 * b + 1] : 1.f;
    // the lane's kernel rows: channel offset, tap shift, validity
    int cof[MT], dr[MT], dc[MT];
    bool rv[MT];
#pragma unroll
    for (int mt = 0; mt < MT; mt++) {
        const int r = r0 + 16 * mt + i16;
        rv[mt] = r < rows;
        const int t = rv[mt] ? r / CI : 0;
        cof[mt] = r - t * CI;
        dr[mt] = TR == 3 ? a.dil * (t / 3 - 1) : 0;
        dc[mt] = TR == 3 ? a.dil * (t % 3 - 1) : 0;
    }
    bool nv[NT];
#pragma unroll
    for (int nt = 0; nt < NT; nt++) nv[nt] = n0 + 16 * nt + i16 < CO;
    const float* xb = a.x + (size_t)b * npx * a.x_cs + a.x_off;
    const float* gm = ln ? a.gamma + a.x_off : nullptr;
    const float* bt = ln ? a.beta + a.x_off : nullptr;
    const int W4 = W >> 2, nsteps = (y1 - y0) * W4;
    const uint32_t m_w4 = udiv_magic(W4);
    const bool do_bias = a.bpart != nullptr && blockIdx.y == 0;
    f4 acc[MT][NT];
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
        for (int nt = 0; nt < NT; nt++) acc[mt][nt] = f4{0.f, 0.f, 0.f, 0.f};
    float bsum[NT];
#pragma unroll
    for (int nt = 0; nt < NT; nt++) bsum[nt] = 0.f;
    // raw operands of step j: x (+ gamma, beta) per kernel row, G per column block. Branch-free and with
    // no select after a load: a lane outside the image (or past CO) reads the zero float a.zero for every
    // operand, so x = gamma = beta = 0 and its A is exactly 0; the next step's loads are issued before
    // this step's MFMAs and waited for only at the next step
    // (buffer loads over the image's range: an out-of-range offset, BUF_OOB for a lane outside the
    // image or past CO, returns 0 — no selects, 32-bit offsets)
    const uint32_t xbytes = (uint32_t)(npx * a.x_cs - a.x_off) * 4u;
    const __amdgpu_buffer_rsrc_t rx = buf_rsrc(xb, xbytes);
    const __amdgpu_buffer_rsrc_t rgm = buf_rsrc(ln ? gm : xb, xbytes), rbt = buf_rsrc(ln ? bt : xb, xbytes);
    const float* gbase = a.dy + (size_t)b * npx * a.dy_cs + a.dy_off;
    const __amdgpu_buffer_rsrc_t rG = buf_rsrc(gbase, (uint32_t)(npx * a.dy_cs - a.dy_off) * 4u);
    float xr[MT], gr[MT], br[MT], gv[NT];
    auto load = [&](int j) {
        const int q = udiv(j, m_w4), yy = y0 + q, xx = 4 * (j - q * W4) + kq;
#pragma unroll
        for (int mt = 0; mt < MT; mt++) {
            const int y = yy + dr[mt], x = xx + dc[mt];
            const bool ok = rv[mt] && (unsigned)y < (unsigned)H && (unsigned)x < (unsigned)W;
            const uint32_t off = ok ? (uint32_t)((y * W + x) * a.x_cs + cof[mt]) * 4u : BUF_OOB;
            xr[mt] = buf_load1(rx, off);
            if (ln) {
                gr[mt] = buf_load1(rgm, off);
                br[mt] = buf_load1(rbt, off);
            }
        }
        const int gi = (yy * W + xx) * a.dy_cs + n0 + i16;
#pragma unroll
        for (int nt = 0; nt < NT; nt++) gv[nt] = buf_load1(rG, nv[nt] ? (uint32_t)(gi + 16 * nt) * 4u : BUF_OOB);
    };
    int j = wave;
    if (j < nsteps) load(j);
    for (; j < nsteps; j += 4) {
        float av[MT], g[NT];
#pragma unroll
        for (int mt = 0; mt < MT; mt++) {
            const float h = act ? lrelu(xr[mt]) : xr[mt];
            av[mt] = ln ? (h - mu) * rs * gr[mt] + br[mt] : h;
        }
#pragma unroll
        for (int nt = 0; nt < NT; nt++) g[nt] = gv[nt];
        if (j + 4 < nsteps) load(j + 4);
#pragma unroll
        for (int mt = 0; mt < MT; mt++)
#pragma unroll
            for (int nt = 0; nt < NT; nt++) acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt], g[nt], acc[mt][nt], 0, 0, 0);
        if (do_bias) {
#pragma unroll
            for (int nt = 0; nt < NT; nt++) bsum[nt] += g[nt];
        }
    }
    // waves 3, 2, 1 add their sums into LDS in that order; wave 0 adds its own and stores the row
    f4* red = reinterpret_cast<f4*>(wdsm);   // [MT * NT][64]
    float* bred = wdsm + MT * NT * 64 * 4;   // [NT][64]
    for (int w = 3; w >= 1; w--) {
        if (wave == w) {
#pragma unroll
            for (int mt = 0; mt < MT; mt++)
#pragma unroll
                for (int nt = 0; nt < NT; nt++) {
                    f4& d = red[(mt * NT + nt) * 64 + lane];
                    d = w == 3 ? acc[mt][nt] : d + acc[mt][nt];
                }
#pragma unroll
            for (int nt = 0; nt < NT; nt++) bred[nt * 64 + lane] = w == 3 ? bsum[nt] : bred[nt * 64 + lane] + bsum[nt];
        }
        __syncthreads();
    }
    if (wave != 0) return;
    float* part = a.part + (size_t)chunk * ((size_t)rows * CO + CO);
#pragma unroll
    for (int mt = 0; mt < MT; mt++)
#pragma unroll
        for (int nt = 0; nt < NT; nt++) {
            const f4 v = red[(mt * NT + nt) * 64 + lane] + acc[mt][nt];
            const int n = n0 + 16 * nt + i16;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int r = r0 + 16 * mt + 4 * kq + q;
                if (r < rows && n < CO) part[(size_t)r * CO + n] = v[q];
            }
        }
    if (do_bias) {
#pragma unroll
        for (int nt = 0; nt < NT; nt++) {
            // lanes i16 + 16 kq hold slices of column n0 + 16 nt + i16: add them in kq order
            float v = bred[nt * 64 + lane] + bsum[nt];
            const float v1 = __shfl(v, i16 + 16), v2 = __shfl(v, i16 + 32), v3 = __shfl(v, i16 + 48);
            v = ((v + v1) + v2) + v3;
            const int n = n0 + 16 * nt + i16;
            if (kq == 0 && n < CO) part[(size_t)rows * CO + n] = v;
        }
    }
}

// k_wgrad_direct's unit split: bands of rows per image so that the launch writes <= WGRAD_MAX_CHUNKS
// partial rows; its tiling: MT row blocks (<= 8) x NT column blocks (<= 4) per workgroup
static void wgrad_direct_shape(const WGradArgs& a, int& RB, int& nbands, int& mt, int& nt, int& gy, int& gz) {
    const int per_img = std::max(1, WGRAD_MAX_CHUNKS / std::max(1, a.B));
    nbands = std::min(a.H, per_img);
    RB = (a.H + nbands - 1) / nbands;
    nbands = (a.H + RB - 1) / RB;
    const int rb = (a.taps * a.CI + 15) / 16, cb = (a.CO + 15) / 16;
    gy = (rb + 7) / 8;
    mt = (rb + gy - 1) / gy;
    gz = (cb + 3) / 4;
    nt = (cb + gz - 1) / gz;
    if (nt == 3) nt = 4;
}

bool wgrad_direct_ok(int H, int W, int taps) { return (W & 3) == 0 && W >= 4 && (taps == 1 || taps == 9); }

int wgrad_direct_chunks(int B, int H) {
    WGradArgs a{};
    a.B = B;
    a.H = H;
    a.W = 4;
    a.taps = 1;
    a.CI = 1;
    a.CO = 1;
    int RB, nb, mt, nt, gy, gz;
    wgrad_direct_shape(a, RB, nb, mt, nt, gy, gz);
    return B * nb;
}

static void launch_wgrad_direct(const WGradArgs& a, hipStream_t st) {
    int RB, nbands, mt, nt, gy, gz;
    wgrad_direct_shape(a, RB, nbands, mt, nt, gy, gz);
    if (a.B * nbands != a.chunks) throw std::logic_error("k_wgrad_direct: chunk count mismatch");
    const dim3 g(a.B * nbands, gy, gz), blk(256);
    const size_t lds = ((size_t)mt * nt * 64 * 4 + (size_t)nt * 64) * 4;
#define CNF_WD(MT_, NT_)                                                                                   \
    if (mt == MT_ && nt == NT_) {                                                                          \
        if (a.taps == 9)                                                                                   \
            hipLaunchKernelGGL((k_wgrad_direct<MT_, NT_, 3>), g, blk, lds, st, a, RB, nbands);              \
        else                                                                                               \
            hipLaunchKernelGGL((k_wgrad_direct<MT_, NT_, 1>), g, blk, lds, st, a, RB, nbands);              \
        return;                                                                                            \
    }
#define CNF_WD_N(MT_) CNF_WD(MT_, 1) CNF_WD(MT_, 2) CNF_WD(MT_, 4)
    CNF_WD_N(1) CNF_WD_N(2) CNF_WD_N(3) CNF_WD_N(4) CNF_WD_N(5) CNF_WD_N(6) CNF_WD_N(7) CNF_WD_N(8)
#undef CNF_WD_N
#undef CNF_WD
    throw std::logic_error("k_wgrad_direct: no instantiation for this tiling");
}

// ------------------------------------------------------------------------------------------------
// k_wgrad_thin: the weight gradient of a 3x3 (dilation 1) convolution with CO <= 4 outputs and
// CI <= 64 inputs (the streamed conv_out: LN_out(LeakyReLU(y)), nk channels -> dc2), where the MFMA
// kernel's 16-wide output tiles are 2/16 used. A workgroup owns TR full rows (<= 128 pixels) of ipw
// images: per image it stages X over the rows and their 1-pixel halo (LN on load, zeros outside) and
// dY in LDS; thread (kh, ci) sums the three taps (kh, 0..2) of input channel ci for every output
// with a sliding window along the row (one LDS read per pixel), CO more threads the bias. One partial
// row [taps][CI][CO] + [CO] per workgroup (<= WGRAD_MAX_CHUNKS), reduced by k_grad_scatter.
// ------------------------------------------------------------------------------------------------
template <int CO>
__global__ __launch_bounds__(256) void k_wgrad_thin(WGradArgs a, int TR, int ipw, int ntile) {
    extern __shared__ __attribute__((aligned(16))) float wsm[];
    const int H = a.H, W = a.W, npx = H * W, CI = a.CI, BW = W + 2, BH = TR + 2, CQ = CI >> 2;
    float* xs = wsm;                          // [BH * BW][CI]
    float* ds = wsm + (size_t)BH * BW * CI;   // [TR * W][CO]
    const int tile = blockIdx.x % ntile, grp = blockIdx.x / ntile;
    const int r0 = tile * TR, nr = min(TR, H - r0);
    const int b0 = grp * ipw, b1 = min(a.B, b0 + ipw);
    const int t = threadIdx.x, ci = t % CI, kh = t / CI;
    const bool wt = t < 3 * CI, bt = t >= 3 * CI && t < 3 * CI + CO;
    float acc[3][CO];
#pragma unroll
    for (int kw = 0; kw < 3; kw++)
#pragma unroll
        for (int co = 0; co < CO; co++) acc[kw][co] = 0.f;
    float bacc = 0.f;
    const bool ln = a.stats != nullptr;
    const int nq = BH * BW * CQ;
    for (int b = b0; b < b1; b++) {
        __syncthreads();   // the previous image's reads are done
        const float mu = ln ? a.stats[2 * b] : 0.f, rs = ln ? a.stats[2 * b + 1] : 1.f;
        // buffer loads (4-byte alignment: x / gamma / beta windows at any float offset; 0 out of range)
        const uint32_t xbytes = (uint32_t)(npx * a.x_cs - a.x_off) * 4u;
        const __amdgpu_buffer_rsrc_t rx = buf_rsrc(a.x + (size_t)b * npx * a.x_cs + a.x_off, xbytes);
        const __amdgpu_buffer_rsrc_t rg = buf_rsrc(ln ? a.gamma + a.x_off : a.x, xbytes);
        const __amdgpu_buffer_rsrc_t rb = buf_rsrc(ln ? a.beta + a.x_off : a.x, xbytes);
        constexpr int U = 8;   // quads per thread and batch (the 32-wide tiles' 3264 quads in two batches)
        for (int e0 = t; e0 < nq; e0 += 256 * U) {
            f4 v[U], g[U], bb[U];
            bool ok[U];
            uint32_t off[U];
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int e = e0 + 256 * u;
                const int pb = e / CQ, q = e - pb * CQ;
                const int br = pb / BW, bc = pb - br * BW;
                const int r = r0 - 1 + br, c = bc - 1;
                ok[u] = e < nq && r >= 0 && r < H && c >= 0 && c < W;
                off[u] = ok[u] ? (uint32_t)((r * W + c) * a.x_cs + 4 * q) * 4u : BUF_OOB;
                v[u] = buf_load4(rx, off[u]);
                if (ln) {
                    g[u] = buf_load4(rg, off[u]);
                    bb[u] = buf_load4(rb, off[u]);
                }
            }
#pragma unroll
            for (int u = 0; u < U; u++) {
                const int e = e0 + 256 * u;
                if (e >= nq) break;
                f4 o;
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float x = v[u][j];
                    const float y = ln ? (lrelu(x) - mu) * rs * g[u][j] + bb[u][j] : (a.act ? lrelu(x) : x);
                    o[j] = ok[u] ? y : 0.f;   // zero padding of the conv input (LN of 0 is not 0)
                }
                *reinterpret_cast<f4*>(xs + 4 * e) = o;
            }
        }
        for (int e = t; e < nr * W * CO; e += 256) {
            const int p = e / CO, co = e - p * CO;
            ds[e] = a.dy[((size_t)b * npx + (size_t)r0 * W + p) * a.dy_cs + a.dy_off + co];
        }
        __syncthreads();
        if (wt) {
            for (int pr = 0; pr < nr; pr++) {
                const float* xr = xs + (size_t)(pr + kh) * BW * CI + ci;
                const float* dr = ds + (size_t)pr * W * CO;
                float x0 = xr[0], x1 = xr[CI];
                for (int pc = 0; pc < W; pc++) {
                    const float x2 = xr[(pc + 2) * CI];
#pragma unroll
                    for (int co = 0; co < CO; co++) {
                        const float d = dr[pc * CO + co];
                        acc[0][co] = fmaf(x0, d, acc[0][co]);
                        acc[1][co] = fmaf(x1, d, acc[1][co]);
                        acc[2][co] = fmaf(x2, d, acc[2][co]);
                    }
                    x0 = x1;
                    x1 = x2;
                }
            }
        } else if (bt) {
            const int co = t - 3 * CI;
            for (int p = 0; p < nr * W; p++) bacc += ds[p * CO + co];
        }
    }
    float* part = a.part + (size_t)blockIdx.x * (9 * CI * CO + CO);
    if (wt)
#pragma unroll
        for (int kw = 0; kw < 3; kw++)
#pragma unroll
            for (int co = 0; co < CO; co++) part[((kh * 3 + kw) * CI + ci) * CO + co] = acc[kw][co];
    if (bt) part[9 * CI * CO + (t - 3 * CI)] = bacc;
}

static void wgrad_thin_shape(int B, int H, int W, int& TR, int& ipw, int& ntile) {
    TR = std::max(1, std::min(H, 128 / std::max(1, W)));
    ntile = (H + TR - 1) / TR;
    ipw = (B * ntile + WGRAD_MAX_CHUNKS - 1) / WGRAD_MAX_CHUNKS;
    if (ipw < 1) ipw = 1;
}

bool wgrad_thin_ok(int H, int W, int taps, int dil, int CI, int CO) {
    const bool on = (opts().train_alt & 8) == 0;   // debug option TRAIN_ALT bit 8: k_wgrad_direct / k_wgrad_band take them
    if (!on || taps != 9 || dil != 1 || CO < 1 || CO > 4 || CI < 4 || CI > 64 || (CI & 3) != 0 || W < 1 || W > 128)
        return false;
    int TR, ipw, ntile;
    wgrad_thin_shape(1, H, W, TR, ipw, ntile);
    return ((size_t)(TR + 2) * (W + 2) * CI + (size_t)TR * W * CO) * 4 <= 64 * 1024;
}

int wgrad_thin_chunks(int B, int H, int W) {
    int TR, ipw, ntile;
    wgrad_thin_shape(B, H, W, TR, ipw, ntile);
    return ntile * ((B + ipw - 1) / ipw);
}

void launch_wgrad_thin(const WGradArgs& a, hipStream_t st) {
    int TR, ipw, ntile;
    wgrad_thin_shape(a.B, a.H, a.W, TR, ipw, ntile);
    if (a.chunks != ntile * ((a.B + ipw - 1) / ipw)) throw std::logic_error("k_wgrad_thin: chunk count mismatch");
    const size_t lds = ((size_t)(TR + 2) * (a.W + 2) * a.CI + (size_t)TR * a.W * a.CO) * 4;
    const dim3 g(a.chunks), blk(256);
    switch (a.CO) {
        case 1: hipLaunchKernelGGL((k_wgrad_thin<1>), g, blk, lds, st, a, TR, ipw, ntile); break;
        case 2: hipLaunchKernelGGL((k_wgrad_thin<2>), g, blk, lds, st, a, TR, ipw, ntile); break;
        case 3: hipLaunchKernelGGL((k_wgrad_thin<3>), g, blk, lds, st, a, TR, ipw, ntile); break;
        case 4: hipLaunchKernelGGL((k_wgrad_thin<4>), g, blk, lds, st, a, TR, ipw, ntile); break;
        default: throw std::invalid_argument("k_wgrad_thin: CO out of range");
    }
}

// rows per work unit (about 128 pixels) and the unit count of a wgrad launch
static void wgrad_units(const WGradArgs& a, int& RB, int& nunits) {
    RB = a.W >= 128 ? 1 : 128 / a.W;
    if (RB > a.H) RB = a.H;
    if (RB < 1) RB = 1;
    nunits = a.B * ((a.H + RB - 1) / RB);
}

int wgrad_band_chunks(int B, int H, int W, int taps, int CI, int CO) {
    WGradArgs a{};
    a.B = B;
    a.H = H;
    a.W = W;
    int RB, nunits;
    wgrad_units(a, RB, nunits);
    const int blocks = ((CI + 63) / 64) * ((CO + 63) / 64) * (taps == 9 ? 3 : 1);
    int c = (768 + blocks - 1) / blocks;   // three 4-wave workgroups per CU
    if (c > WGRAD_MAX_CHUNKS) c = WGRAD_MAX_CHUNKS;
    if (c > nunits) c = nunits;
    return c < 1 ? 1 : c;
}

size_t wgrad_band_lds(int H, int W, int taps, int dil, int CI, int CO) {
    WGradArgs a{};
    a.B = 1;
    a.H = H;
    a.W = W;
    int RB, nunits;
    wgrad_units(a, RB, nunits);
    const int hx = taps == 9 ? dil : 0;
    const int CIB = CI < 64 ? CI : 64, COB = CO < 64 ? CO : 64;
    const size_t stage = ((size_t)RB * (W + 2 * hx) * wg_stride(CIB) + (size_t)((RB * W + 3) & ~3) * wg_stride(COB)) * 4;
    const size_t red = CIB <= 32 ? (size_t)4 * (taps == 9 ? 3 : 1) * 16 * 64 * 4 : 0;   // k-slice sums
    return stage > red ? stage : red;
}

bool wgrad_band_ok(int H, int W, int taps, int dil, int CI, int CO) {
    return (taps == 1 || taps == 9) && W >= 4 && wgrad_band_lds(H, W, taps, dil, CI, CO) <= 160 * 1024;
}

void launch_wgrad(const WGradArgs& a, hipStream_t st) {
    if (a.chunk_px == -1) {   // k_wgrad_direct (the caller checked wgrad_direct_ok and sized chunks)
        launch_wgrad_direct(a, st);
        return;
    }
    if (a.chunk_px > 0) {   // k_wgrad, the VALU kernel: the caller chose it (CNF_TRAIN_VALU, or !wgrad_band_ok)
        const dim3 g(a.chunks, a.taps, ((a.CI + 63) / 64) * ((a.CO + 63) / 64)), blk(256);
        hipLaunchKernelGGL(k_wgrad, g, blk, 0, st, a);
        return;
    }
    if (a.taps != 1 && a.taps != 9) throw std::invalid_argument("k_wgrad_band: taps must be 1 or 9");
    if (a.W < 4) throw std::invalid_argument("k_wgrad_band: image width below 4");
    int RB, nunits;
    wgrad_units(a, RB, nunits);
    const size_t lds = wgrad_band_lds(a.H, a.W, a.taps, a.dil, a.CI, a.CO);
    if (lds > 160 * 1024) throw std::invalid_argument("k_wgrad_band: band exceeds the LDS budget");
    const dim3 g(a.chunks, a.taps == 9 ? 3 : 1, ((a.CI + 63) / 64) * ((a.CO + 63) / 64)), blk(256);
    if (a.taps == 9)
        hipLaunchKernelGGL(k_wgrad_band<3>, g, blk, lds, st, a, RB, nunits);
    else
        hipLaunchKernelGGL(k_wgrad_band<1>, g, blk, lds, st, a, RB, nunits);
}

// 32 elements per workgroup (one 128-byte line of a partial row per half-wave), 32 slices of the
// chunk rows per element, every load of a slice in flight at once (<= 8 per thread up to 256 chunks),
// then a fixed-order LDS sum over the slices: deterministic
constexpr int GS_EL = 32, GS_SL = 32, GS_U = 8;
__global__ __launch_bounds__(GS_EL * GS_SL) void k_grad_scatter(const float* __restrict__ part, int chunks, long long n,
                                                                const int64_t* __restrict__ map, float* __restrict__ dparams) {
    __shared__ double red[GS_SL][GS_EL];
    const int t = threadIdx.x, el = t & (GS_EL - 1), sl = t / GS_EL;
    const long long i = (long long)blockIdx.x * GS_EL + el;
    // the destination and its current value are fetched first, behind the partial-row loads (only this
    // launch writes these parameters' gradients)
    int64_t dst = -1;
    float old = 0.f;
    if (sl == 0 && i < n) {
        dst = map[i];
        if (dst >= 0) old = dparams[dst];
    }
    double s = 0.0;
    if (i < n) {
        for (int c0 = sl; c0 < chunks; c0 += GS_SL * GS_U) {
            float v[GS_U];
#pragma unroll
            for (int u = 0; u < GS_U; u++) {
                const int c = c0 + GS_SL * u;
                v[u] = c < chunks ? part[(size_t)c * n + i] : 0.f;
            }
#pragma unroll
            for (int u = 0; u < GS_U; u++) s += (double)v[u];
        }
    }
    red[sl][el] = s;
    __syncthreads();
    if (sl == 0 && i < n) {
        double tot = 0.0;
#pragma unroll
        for (int k = 0; k < GS_SL; k++) tot += red[k][el];
        if (dst >= 0) dparams[dst] = old + (float)tot;
    }
}

void launch_grad_scatter(const float* part, int chunks, long long n, const int64_t* map, float* dparams, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_grad_scatter, dim3((unsigned)((n + GS_EL - 1) / GS_EL)), dim3(GS_EL * GS_SL), 0, st, part, chunks, n, map,
                       dparams);
}

// ------------------------------------------------------------------------------------------------
// LayerNorm (over H*W*C per image, keras epsilon 1e-3, biased variance) of LeakyReLU(x)
// ------------------------------------------------------------------------------------------------
// One 1024-thread workgroup per image: float4 loads, four in flight per thread and pass, fp64
// accumulation (the per-image reductions are latency-bound otherwise: one dependent load per
// thread and step).
constexpr int LNT = 1024;

__device__ __forceinline__ double block_sum_ln(double v, double* red) {
    v = wave_sum(v);
    __syncthreads();
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < LNT / 64; w++) t += red[w];
    return t;
}

__global__ __launch_bounds__(LNT) void k_ln_stats(const float* __restrict__ x, long long n, int act,
                                                  float* __restrict__ stats) {
    __shared__ double red[LNT / 64];
    const int b = blockIdx.x;
    const float* xb = x + (size_t)b * n;
    double s1 = 0.0, s2 = 0.0;
    if ((n & 3) == 0) {
        const f4* x4 = reinterpret_cast<const f4*>(xb);
        const long long n4 = n >> 2;
        for (long long i0 = threadIdx.x; i0 < n4; i0 += 4LL * LNT) {
            f4 v[4];
#pragma unroll
            for (int u = 0; u < 4; u++) v[u] = i0 + u * LNT < n4 ? x4[i0 + u * LNT] : f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int u = 0; u < 4; u++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const double h = act ? lrelu(v[u][j]) : v[u][j];
                    s1 += h;
                    s2 += h * h;
                }
        }
    } else {
        for (long long e = threadIdx.x; e < n; e += LNT) {
            const double h = act ? lrelu(xb[e]) : xb[e];
            s1 += h;
            s2 += h * h;
        }
    }
    s1 = block_sum_ln(s1, red);
    s2 = block_sum_ln(s2, red);
    if (threadIdx.x == 0) {
        const double m = s1 / (double)n;
        double var = s2 / (double)n - m * m;
        if (var < 0.0) var = 0.0;
        stats[2 * b] = (float)m;
        stats[2 * b + 1] = (float)(1.0 / sqrt(var + (double)LN_EPS));
    }
}

void launch_ln_stats(const float* x, long long n, int B, int act, float* stats, hipStream_t st) {
    hipLaunchKernelGGL(k_ln_stats, dim3(B), dim3(LNT), 0, st, x, n, act, stats);
}

// per image: sums[b] = (sum g, sum g*xhat), g = dxo * gamma
__global__ __launch_bounds__(LNT) void k_lnb_reduce(const float* __restrict__ x, const float* __restrict__ dxo,
                                                    const float* __restrict__ gamma, const float* __restrict__ stats,
                                                    long long n, double* __restrict__ sums, unsigned long long cmask,
                                                    int cmod) {
    __shared__ double red[LNT / 64];
    // channel mask (cmod > 0): elements of unset channels count as dxo = 0
    auto live = [&](long long e) { return cmod == 0 || ((cmask >> ((uint32_t)e % (uint32_t)cmod)) & 1ull) != 0; };
    const int b = blockIdx.x, sl = blockIdx.y, RS = gridDim.y;   // slice sl of image b's elements
    const float* xb = x + (size_t)b * n;
    const float* db = dxo + (size_t)b * n;
    const float mu = stats[2 * b], rs = stats[2 * b + 1];
    double sg = 0.0, sgh = 0.0;
    if ((n & 3) == 0 && (reinterpret_cast<uintptr_t>(gamma) & 15) == 0) {
        const long long n4 = n >> 2, q = (n4 + RS - 1) / RS, lo = sl * q, hi = min(n4, lo + q);
        const f4* x4 = reinterpret_cast<const f4*>(xb);
        const f4* d4 = reinterpret_cast<const f4*>(db);
        const f4* g4 = reinterpret_cast<const f4*>(gamma);
        for (long long i0 = lo + threadIdx.x; i0 < hi; i0 += 2LL * LNT) {
            f4 xv[2], dv[2], gv[2];
#pragma unroll
            for (int u = 0; u < 2; u++) {
                const long long i = i0 + u * LNT;
                const bool ok = i < hi;
                xv[u] = ok ? x4[i] : f4{0.f, 0.f, 0.f, 0.f};
                dv[u] = ok ? d4[i] : f4{0.f, 0.f, 0.f, 0.f};
                gv[u] = ok ? g4[i] : f4{0.f, 0.f, 0.f, 0.f};
                if (cmod != 0)
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (!live(4 * i + j)) dv[u][j] = 0.f;
            }
#pragma unroll
            for (int u = 0; u < 2; u++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float xh = (lrelu(xv[u][j]) - mu) * rs;
                    const float g = dv[u][j] * gv[u][j];
                    sg += g;
                    sgh += (double)g * xh;
                }
        }
    } else {
        const long long q = (n + RS - 1) / RS, lo = sl * q, hi = min(n, lo + q);
        for (long long e = lo + threadIdx.x; e < hi; e += LNT) {
            const float xh = (lrelu(xb[e]) - mu) * rs;
            const float g = (live(e) ? db[e] : 0.f) * gamma[e];
            sg += g;
            sgh += (double)g * xh;
        }
    }
    sg = block_sum_ln(sg, red);
    sgh = block_sum_ln(sgh, red);
    if (threadIdx.x == 0) {
        sums[2 * ((size_t)b * RS + sl)] = sg;
        sums[2 * ((size_t)b * RS + sl) + 1] = sgh;
    }
}

// four consecutive elements per lane (one float4), over the images of batch slice blockIdx.y (four
// at a time, their loads in flight together): dx, and the slice's dgamma / dbeta partials summed in
// registers; k_lnb_gsum adds the slices in a fixed order (no atomics: deterministic)
constexpr int LNA_MAXIMG = 256;   // images per batch slice whose sums k_lnb_apply shares through LDS
__global__ __launch_bounds__(256) void k_lnb_apply(const float* __restrict__ x, const float* __restrict__ dxo,
                                                   const float* __restrict__ gamma, const float* __restrict__ stats,
                                                   const double* __restrict__ sums, int rsl, int rstride, long long n,
                                                   int B, int act,
                                                   float* __restrict__ dx, int accumulate, float* __restrict__ gpart,
                                                   float* __restrict__ bpart, unsigned long long cmask, int cmod) {
    const long long e0 = ((long long)blockIdx.x * 256 + threadIdx.x) * 4;
    const int S = gridDim.y, sl = blockIdx.y;
    const int bs = (B + S - 1) / S, b_lo = sl * bs, b_hi = min(B, b_lo + bs);
    const float inv_n0 = 1.f / (float)n;
    // the slice's per-image means of g and g * xhat, summed once per workgroup (one thread per image, its
    // partials in order) instead of by every thread
    __shared__ float smg[LNA_MAXIMG], smgh[LNA_MAXIMG];
    const bool shared_sums = stats != nullptr && b_hi - b_lo <= LNA_MAXIMG;
    if (shared_sums) {
        const int b = b_lo + (int)threadIdx.x;
        if (b < b_hi) {
            double s0 = 0.0, s1 = 0.0;
            for (int k = 0; k < rsl; k++) {
                s0 += sums[2 * ((size_t)b * rstride + k)];
                s1 += sums[2 * ((size_t)b * rstride + k) + 1];
            }
            smg[threadIdx.x] = (float)(s0 * inv_n0);
            smgh[threadIdx.x] = (float)(s1 * inv_n0);
        }
        __syncthreads();
    }
    if (e0 >= n) return;
    const bool vec = (n & 3) == 0;
    const int ne = n - e0 < 4 ? (int)(n - e0) : 4;
    f4 gm = f4{1.f, 1.f, 1.f, 1.f}, dg = f4{0.f, 0.f, 0.f, 0.f}, dbt = f4{0.f, 0.f, 0.f, 0.f};
    if (stats)
        for (int j = 0; j < ne; j++) gm[j] = gamma[e0 + j];
    const float inv_n = 1.f / (float)n;
    auto ld4 = [&](const float* p, size_t i) -> f4 {
        if (vec) return *reinterpret_cast<const f4*>(p + i);
        f4 v = f4{0.f, 0.f, 0.f, 0.f};
        for (int j = 0; j < ne; j++) v[j] = p[i + j];
        return v;
    };
    // channel mask (cmod > 0): the lane's elements of unset channels are dxo = 0 (not loaded)
    f4 dm = f4{1.f, 1.f, 1.f, 1.f};
    if (cmod != 0)
        for (int j = 0; j < 4; j++) dm[j] = ((cmask >> ((uint32_t)(e0 + j) % (uint32_t)cmod)) & 1ull) ? 1.f : 0.f;
    const bool dld = dm[0] != 0.f || dm[1] != 0.f || dm[2] != 0.f || dm[3] != 0.f;
    constexpr int U = 4;
    for (int b0 = b_lo; b0 < b_hi; b0 += U) {
        f4 xv[U], d[U], o[U];
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int b = b0 + u;
            const size_t i = (size_t)b * n + e0;
            xv[u] = b < b_hi ? ld4(x, i) : f4{0.f, 0.f, 0.f, 0.f};
            d[u] = b < b_hi && dld ? ld4(dxo, i) : f4{0.f, 0.f, 0.f, 0.f};
            if (cmod != 0)
#pragma unroll
                for (int j = 0; j < 4; j++) d[u][j] = dm[j] != 0.f ? d[u][j] : 0.f;
            o[u] = (accumulate && b < b_hi) ? ld4(dx, i) : f4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < U; u++) {
            const int b = b0 + u;
            if (b >= b_hi) break;
            float mu = 0.f, rs = 1.f, mg = 0.f, mgh = 0.f;
            if (stats) {
                mu = stats[2 * b];
                rs = stats[2 * b + 1];
                if (shared_sums) {
                    mg = smg[b - b_lo];
                    mgh = smgh[b - b_lo];
                } else {
                    double s0 = 0.0, s1 = 0.0;   // the image's slice partials, in slice order
                    for (int k = 0; k < rsl; k++) {
                        s0 += sums[2 * ((size_t)b * rstride + k)];
                        s1 += sums[2 * ((size_t)b * rstride + k) + 1];
                    }
                    mg = (float)(s0 * inv_n);
                    mgh = (float)(s1 * inv_n);
                }
            }
            f4 g4;
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float lr = (!act || xv[u][j] > 0.f) ? 1.f : LRELU_ALPHA;
                float g;
                if (stats) {
                    const float xh = (lrelu(xv[u][j]) - mu) * rs;
                    dg[j] = fmaf(d[u][j], xh, dg[j]);
                    dbt[j] += d[u][j];
                    g = rs * (d[u][j] * gm[j] - mg - xh * mgh) * lr;
                } else {
                    g = d[u][j] * lr;
                }
                g4[j] = o[u][j] + g;
            }
            const size_t i = (size_t)b * n + e0;
            if (vec) {
                *reinterpret_cast<f4*>(dx + i) = g4;
            } else {
                for (int j = 0; j < ne; j++) dx[i + j] = g4[j];
            }
        }
    }
    if (stats)
        for (int j = 0; j < ne; j++) {
            gpart[(size_t)sl * n + e0 + j] = dg[j];
            bpart[(size_t)sl * n + e0 + j] = dbt[j];
        }
}

__global__ __launch_bounds__(256) void k_lnb_gsum(const float* __restrict__ gpart, const float* __restrict__ bpart,
                                                  int S, long long n, float* __restrict__ dgamma,
                                                  float* __restrict__ dbeta) {
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    float g = 0.f, b = 0.f;
    for (int s = 0; s < S; s++) {
        g += gpart[(size_t)s * n + e];
        b += bpart[(size_t)s * n + e];
    }
    dgamma[e] += g;
    dbeta[e] += b;
}

void launch_ln_backward(const float* x, const float* dxo, const float* gamma, const float* stats, double* sums,
                        long long n, int B, int act, float* dx, int accumulate, float* dgamma, float* dbeta,
                        float* scratch, hipStream_t st, int presum, int pstride, unsigned long long cmask, int cmod) {
    if (cmod < 0 || cmod > 64) throw std::invalid_argument("launch_ln_backward: channel mask over <= 64 channels");
    // slices per image: at least two full passes of the workgroup each (64 images x 8 slices fill the
    // GPU where one workgroup per image used a quarter of it)
#ifndef CNF_LNB_RS
#define CNF_LNB_RS LNB_RS
#endif
    int rsl = (int)std::min<long long>(CNF_LNB_RS, std::max<long long>(1, (n / 4) / (2LL * LNT)));
    int rstride = rsl;
    if (presum > 0) {
        rsl = presum;
        rstride = pstride > 0 ? pstride : presum;
    } else if (stats)
        hipLaunchKernelGGL(k_lnb_reduce, dim3(B, rsl), dim3(LNT), 0, st, x, dxo, gamma, stats, n, sums, cmask, cmod);
    const int S = B < LNB_SLICES ? B : LNB_SLICES;
    float* gpart = scratch;
    float* bpart = scratch + (size_t)LNB_SLICES * n;
    hipLaunchKernelGGL(k_lnb_apply, dim3((unsigned)((n + 1023) / 1024), S), dim3(256), 0, st, x, dxo, gamma, stats,
                       sums, rsl, rstride, n, B, act, dx, accumulate, gpart, bpart, cmask, cmod);
    if (stats)
        hipLaunchKernelGGL(k_lnb_gsum, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, gpart, bpart, S, n, dgamma,
                           dbeta);
}

// ------------------------------------------------------------------------------------------------
// affine coupling backward (forward law :1076-1213 / k_coupling): v1 = u1, v2 = exp(s) u2 + t,
// s = w tanh(a), per-image log-det sum s
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_coup_bw(CoupBwArgs a) {
    __shared__ double red[4];
    const int img = blockIdx.y;
    const int HWD = a.H * a.W * a.D, npx = a.hc * a.wc;
    const float* ub = a.u + (size_t)img * HWD;
    const float* dvb = a.dv + (size_t)img * HWD;
    float* dub = a.du + (size_t)img * HWD;
    const float* sb = a.s_pre + (size_t)img * npx * a.dc2;
    float* dsb = a.ds_pre + (size_t)img * npx * a.dc2;
    float* dtb = a.dt + (size_t)img * npx * a.dc2;
    const float w = *a.tanh_w;
    const float g_ld = a.count != nullptr ? -(float)(1.0 / (double)*a.count) : a.g_ld;
    double dw = 0.0;
    for (int p = blockIdx.x * 256 + threadIdx.x; p < npx; p += gridDim.x * 256) {
        for (int c = 0; c < a.dc1; c++) {
            const int e = mask_pos(a.mask, p, c, a.wc, a.W, a.D);
            dub[e] = dvb[e];
        }
        for (int c = 0; c < a.dc2; c++) {
            const int e = mask_pos(a.mask_c, p, c, a.wc, a.W, a.D);
            const int q = p * a.dc2 + c;
            const float th = cpl_tanh(sb[q]);
            const float ex = cpl_exp(w * th);
            const float g = dvb[e];
            dub[e] = g * ex;
            const float ds = g * ex * ub[e] + g_ld;
            dsb[q] = ds * w * (1.f - th * th);
            dtb[q] = g;
            dw += (double)ds * th;
        }
    }
    dw = block_sum256(dw, red);
    if (threadIdx.x == 0) a.dw_part[(size_t)img * gridDim.x + blockIdx.x] = dw;
}

void launch_coupling_backward(const CoupBwArgs& a, int B, int nparts, hipStream_t st) {
    hipLaunchKernelGGL(k_coup_bw, dim3(nparts, B), dim3(256), 0, st, a);
}

__global__ __launch_bounds__(256) void k_scatter_add_u1c(const float* __restrict__ du1c, float* __restrict__ du, int H,
                                                         int W, int D, int mask, int hc, int wc, int dc1) {
    const int img = blockIdx.y;
    const int n = hc * wc * dc1;
    float* ob = du + (size_t)img * H * W * D;
    const float* ib = du1c + (size_t)img * n;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
        const int p = e / dc1, c = e - p * dc1;
        ob[mask_pos(mask, p, c, wc, W, D)] += ib[e];
    }
}

void launch_scatter_add_u1c(const float* du1c, float* du, int B, int H, int W, int D, int mask, int hc, int wc, int dc1,
                            hipStream_t st) {
    int n = hc * wc * dc1;
    int gx = (n + 255) / 256;
    if (gx > 64) gx = 64;
    hipLaunchKernelGGL(k_scatter_add_u1c, dim3(gx, B), dim3(256), 0, st, du1c, du, H, W, D, mask, hc, wc, dc1);
}

__global__ void k_dsum(const double* __restrict__ part, long long n, float* __restrict__ out) {
    double s = 0.0;
    for (long long i = threadIdx.x; i < n; i += 64) s += part[i];
    s = wave_sum(s);
    if (threadIdx.x == 0) *out += (float)s;
}

void launch_dsum(const double* part, long long n, float* out, hipStream_t st) {
    hipLaunchKernelGGL(k_dsum, dim3(1), dim3(64), 0, st, part, n, out);
}

// loss = -(mean_b(llz + lly) + mean_b(logdet)) over the global batch (inv_batch = 1 / global B)
__global__ __launch_bounds__(256) void k_nll_grad(const float* __restrict__ xy, const float* __restrict__ zy,
                                                  float* __restrict__ dzy, long long total, int D, int x_d,
                                                  float lambda_y, float inv_batch_h, const float* __restrict__ count) {
    const float inv_batch = count != nullptr ? (float)(1.0 / (double)*count) : inv_batch_h;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        const int c = (int)(e % D);
        const float z = zy[e];
        float g;
        if (c < x_d) {
            g = z * inv_batch;
        } else {
            const float d = z - xy[e];
            g = (d > 0.f ? lambda_y : d < 0.f ? -lambda_y : 0.f) * inv_batch;
        }
        dzy[e] = g;
    }
}

void launch_nll_grad(const float* xy, const float* zy, float* dzy, int B, int HW, int D, int x_d, float lambda_y,
                     float inv_batch, const float* count, hipStream_t st) {
    const long long total = (long long)B * HW * D;
    long long gx = (total + 255) / 256;
    if (gx > 8192) gx = 8192;
    hipLaunchKernelGGL(k_nll_grad, dim3((unsigned)gx), dim3(256), 0, st, xy, zy, dzy, total, D, x_d, lambda_y,
                       inv_batch, count);
}

// Keras Adam (optimizer.Adam: m += (g - m)(1 - b1); v += (g^2 - v)(1 - b2);
// p -= alpha m / (sqrt(v) + eps), alpha = lr sqrt(1 - b2^t) / (1 - b1^t))
__global__ __launch_bounds__(256) void k_adam(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                              float* __restrict__ v, long long n, float alpha, float b1, float b2,
                                              float eps) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const float gi = g[i];
        const float mi = m[i] + (gi - m[i]) * (1.f - b1);
        const float vi = v[i] + (gi * gi - v[i]) * (1.f - b2);
        m[i] = mi;
        v[i] = vi;
        p[i] -= alpha * mi / (sqrtf(vi) + eps);
    }
}

void launch_adam(float* params, const float* grads, float* m, float* v, long long n, float alpha, float b1, float b2,
                 float eps, hipStream_t st) {
    long long gx = (n + 255) / 256;
    if (gx > 8192) gx = 8192;
    if (gx < 1) gx = 1;
    hipLaunchKernelGGL(k_adam, dim3((unsigned)gx), dim3(256), 0, st, params, grads, m, v, n, alpha, b1, b2, eps);
}

}  // namespace cnf
