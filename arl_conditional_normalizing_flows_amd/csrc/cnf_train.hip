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
#include <cstdlib>

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
template <int NR, bool VEC>
__global__ __launch_bounds__(256) void k_tconv_mfma(TConvArgs a) {
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
    f4 acc[NR];
#pragma unroll
    for (int m = 0; m < NR; m++) acc[m] = f4{0.f, 0.f, 0.f, 0.f};
    const int nw = G * 16 * NS;
    for (int tap = 0; tap < a.taps; tap++) {
        const int dr = a.taps == 1 ? 0 : tap / 3 - 1, dc = a.taps == 1 ? 0 : tap % 3 - 1;
        const int r = pr + a.sgn * a.dil * dr, c = pc + a.sgn * a.dil * dc;
        const bool sv = pav && r >= 0 && r < a.H && c >= 0 && c < a.W;
        const size_t q = sv ? (size_t)r * a.W + c : 0;
        __syncthreads();   // the previous tap's B reads are done
        for (int e = threadIdx.x; e < nw; e += 256) {
            const int s4 = e & 3, j = (e >> 2) % NS, gq = (e >> 2) / NS;   // gq = 4g + kq'
            const int k = 4 * gq + s4, n = n0 + j;
            wsm[e] = (k < a.K && n < a.N) ? a.w[tap * a.wt + (long long)k * a.wk + (long long)n * a.wn] : 0.f;
        }
        __syncthreads();
        for (int g = 0; g < G; g++) {
            const int k0 = 16 * g + 4 * kq;
            f4 x = f4{0.f, 0.f, 0.f, 0.f};
            if (sv) {
                const size_t gi = q * a.in_cs + k0;
                if (VEC) {
                    if (k0 < a.K) {
                        x = *reinterpret_cast<const f4*>(inb + gi);
                        if (ln) {
                            const f4 gm = *reinterpret_cast<const f4*>(a.gamma + a.in_off + gi);
                            const f4 bt = *reinterpret_cast<const f4*>(a.beta + a.in_off + gi);
#pragma unroll
                            for (int j = 0; j < 4; j++) x[j] = (lrelu(x[j]) - mu) * rs * gm[j] + bt[j];
                        } else if (a.act) {
#pragma unroll
                            for (int j = 0; j < 4; j++) x[j] = lrelu(x[j]);
                        }
                    }
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++)
                        if (k0 + j < a.K) x[j] = act_load(inb[gi + j], a.act, a.stats, a.gamma, a.beta, b, a.in_off + gi + j);
                }
            }
            const f4* bw = reinterpret_cast<const f4*>(wsm) + (size_t)(4 * g + kq) * NS + i16;
#pragma unroll
            for (int m = 0; m < NR; m++) {
                const f4 bv = bw[16 * m];
#pragma unroll
                for (int s = 0; s < 4; s++) acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(x[s], bv[s], acc[m], 0, 0, 0);
            }
        }
    }
    // acc[m][rr] = out[pixel p0 + 16 wave + 4 kq + rr][channel n0 + 16 m + i16]
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
        }
    }
}

static bool train_valu() {
    static const bool v = [] {   // A/B knob: the register-blocked VALU kernels
        const char* e = std::getenv("CNF_TRAIN_VALU");
        return e && std::atoi(e) != 0;
    }();
    return v;
}

void launch_tconv(const TConvArgs& a, hipStream_t st) {
    const int npx = a.H * a.W;
    if (!train_valu()) {
        const int nr = a.N <= 16 ? 1 : a.N <= 32 ? 2 : a.N <= 48 ? 3 : 4;
        const int NS = 16 * nr;
        const int G = (a.K + 15) / 16;
        const size_t lds = (size_t)G * 16 * NS * 4;
        if (lds <= 64 * 1024) {
            const bool vec = a.K % 4 == 0 && a.in_cs % 4 == 0 && a.in_off % 4 == 0;
            const dim3 g((npx + 63) / 64, a.B, (a.N + NS - 1) / NS), blk(256);
#define CNF_TM(NR_)                                                                                   \
    if (nr == NR_) {                                                                                  \
        if (vec)                                                                                      \
            hipLaunchKernelGGL((k_tconv_mfma<NR_, true>), g, blk, lds, st, a);                      \
        else                                                                                          \
            hipLaunchKernelGGL((k_tconv_mfma<NR_, false>), g, blk, lds, st, a);                     \
        return;                                                                                       \
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
// k_wgrad_mfma: the same weight gradient on v_mfma_f32_16x16x4_f32, a (ci, co) = 64 x 64 tile per
// workgroup, K = the chunk's pixels. Each 32-pixel step stages X (LN-on-load, shifted by the tap)
// and dY into LDS (the next step's values are loaded into registers behind this step's MFMAs);
// wave w owns ci rows 16w.. of the tile: lane (i16, kq) feeds X[px 4s+kq][ci 16w+i16] and
// dY[px 4s+kq][co 16m+i16], so acc[m][r] = dW[ci 16w+4kq+r][co 16m+i16].
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_wgrad_mfma(WGradArgs a) {
    constexpr int SP = 32, XS = 80, NE = SP * 64 / 256;   // row stride 80: conflict-free half-wave reads
    __shared__ __attribute__((aligned(16))) float Xs[SP * XS];
    __shared__ __attribute__((aligned(16))) float Ds[SP * XS];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, i16 = lane & 15, kq = lane >> 4;
    const int npx = a.H * a.W;
    const long long total = (long long)a.B * npx;
    const int tap = blockIdx.y;
    const int nco = (a.CO + 63) / 64;
    const int ci0 = (blockIdx.z / nco) * 64, co0 = (blockIdx.z % nco) * 64;
    const int dr = a.taps == 1 ? 0 : tap / 3 - 1, dc = a.taps == 1 ? 0 : tap % 3 - 1;
    const long long g0 = (long long)blockIdx.x * a.chunk_px;
    const long long g1 = g0 + a.chunk_px < total ? g0 + a.chunk_px : total;
    const bool do_bias = a.bpart != nullptr && tap == 0 && ci0 == 0;
    f4 acc[4];
#pragma unroll
    for (int m = 0; m < 4; m++) acc[m] = f4{0.f, 0.f, 0.f, 0.f};
    float bacc = 0.f;
    float xv[NE], dv[NE];
    auto load = [&](long long gs) {
#pragma unroll
        for (int u = 0; u < NE; u++) {
            const int e = t + 256 * u;
            const int c = e & 63, px = e >> 6;
            const long long g = gs + px;
            float x = 0.f, d = 0.f;
            if (g < g1) {
                const int b = (int)(g / npx), p = (int)(g - (long long)b * npx);
                if (co0 + c < a.CO) d = a.dy[((size_t)b * npx + p) * a.dy_cs + a.dy_off + co0 + c];
                if (ci0 + c < a.CI) {
                    const int r = p / a.W + a.dil * dr, cc = p % a.W + a.dil * dc;
                    if (r >= 0 && r < a.H && cc >= 0 && cc < a.W) {
                        const size_t q = (size_t)r * a.W + cc;
                        const size_t gi = q * a.x_cs + a.x_off + ci0 + c;
                        x = act_load(a.x[(size_t)b * npx * a.x_cs + gi], a.act, a.stats, a.gamma, a.beta, b, gi);
                    }
                }
            }
            xv[u] = x;
            dv[u] = d;
        }
    };
    load(g0);
    for (long long gs = g0; gs < g1; gs += SP) {
        __syncthreads();   // the previous step's LDS reads are done
#pragma unroll
        for (int u = 0; u < NE; u++) {
            const int e = t + 256 * u;
            Xs[(e >> 6) * XS + (e & 63)] = xv[u];
            Ds[(e >> 6) * XS + (e & 63)] = dv[u];
        }
        __syncthreads();
        if (gs + SP < g1) load(gs + SP);   // in flight during this step's MFMAs
#pragma unroll
        for (int s = 0; s < SP / 4; s++) {
            const int px = 4 * s + kq;
            const float av = Xs[px * XS + 16 * wave + i16];
#pragma unroll
            for (int m = 0; m < 4; m++)
                acc[m] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, Ds[px * XS + 16 * m + i16], acc[m], 0, 0, 0);
        }
        if (do_bias && t < 64) {
#pragma unroll
            for (int px = 0; px < SP; px++) bacc += Ds[px * XS + t];
        }
    }
    float* part = a.part + (size_t)blockIdx.x * a.taps * a.CI * a.CO;
#pragma unroll
    for (int r = 0; r < 4; r++) {
        const int ci = ci0 + 16 * wave + 4 * kq + r;
        if (ci >= a.CI) continue;
#pragma unroll
        for (int m = 0; m < 4; m++) {
            const int co = co0 + 16 * m + i16;
            if (co < a.CO) part[((size_t)tap * a.CI + ci) * a.CO + co] = acc[m][r];
        }
    }
    if (do_bias && t < 64 && co0 + t < a.CO) a.bpart[(size_t)blockIdx.x * a.CO + co0 + t] = bacc;
}

void launch_wgrad(const WGradArgs& a, hipStream_t st) {
    const dim3 g(a.chunks, a.taps, ((a.CI + 63) / 64) * ((a.CO + 63) / 64)), blk(256);
    if (train_valu())
        hipLaunchKernelGGL(k_wgrad, g, blk, 0, st, a);
    else
        hipLaunchKernelGGL(k_wgrad_mfma, g, blk, 0, st, a);
}

__global__ __launch_bounds__(256) void k_grad_scatter(const float* __restrict__ part, int chunks, long long n,
                                                      const int64_t* __restrict__ map, float* __restrict__ dparams) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const int64_t dst = map[i];
        if (dst < 0) continue;
        double s = 0.0;
        for (int c = 0; c < chunks; c++) s += (double)part[(size_t)c * n + i];
        dparams[dst] += (float)s;
    }
}

void launch_grad_scatter(const float* part, int chunks, long long n, const int64_t* map, float* dparams, hipStream_t st) {
    long long gx = (n + 255) / 256;
    if (gx > 4096) gx = 4096;
    if (gx < 1) gx = 1;
    hipLaunchKernelGGL(k_grad_scatter, dim3((unsigned)gx), dim3(256), 0, st, part, chunks, n, map, dparams);
}

// ------------------------------------------------------------------------------------------------
// LayerNorm (over H*W*C per image, keras epsilon 1e-3, biased variance) of LeakyReLU(x)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_ln_stats(const float* __restrict__ x, long long n, int act,
                                                  float* __restrict__ stats) {
    __shared__ double red[4];
    const int b = blockIdx.x;
    const float* xb = x + (size_t)b * n;
    double s1 = 0.0, s2 = 0.0;
    for (long long e = threadIdx.x; e < n; e += 256) {
        const double h = act ? lrelu(xb[e]) : xb[e];
        s1 += h;
        s2 += h * h;
    }
    s1 = block_sum256(s1, red);
    s2 = block_sum256(s2, red);
    if (threadIdx.x == 0) {
        const double m = s1 / (double)n;
        double var = s2 / (double)n - m * m;
        if (var < 0.0) var = 0.0;
        stats[2 * b] = (float)m;
        stats[2 * b + 1] = (float)(1.0 / sqrt(var + (double)LN_EPS));
    }
}

void launch_ln_stats(const float* x, long long n, int B, int act, float* stats, hipStream_t st) {
    hipLaunchKernelGGL(k_ln_stats, dim3(B), dim3(256), 0, st, x, n, act, stats);
}

// per image: sums[b] = (sum g, sum g*xhat), g = dxo * gamma
__global__ __launch_bounds__(256) void k_lnb_reduce(const float* __restrict__ x, const float* __restrict__ dxo,
                                                    const float* __restrict__ gamma, const float* __restrict__ stats,
                                                    long long n, double* __restrict__ sums) {
    __shared__ double red[4];
    const int b = blockIdx.x;
    const float* xb = x + (size_t)b * n;
    const float* db = dxo + (size_t)b * n;
    const float mu = stats[2 * b], rs = stats[2 * b + 1];
    double sg = 0.0, sgh = 0.0;
    for (long long e = threadIdx.x; e < n; e += 256) {
        const float xh = (lrelu(xb[e]) - mu) * rs;
        const float g = db[e] * gamma[e];
        sg += g;
        sgh += (double)g * xh;
    }
    sg = block_sum256(sg, red);
    sgh = block_sum256(sgh, red);
    if (threadIdx.x == 0) {
        sums[2 * b] = sg;
        sums[2 * b + 1] = sgh;
    }
}

// one lane per tensor element, looping over the batch: dx, and dgamma / dbeta summed in registers
__global__ __launch_bounds__(256) void k_lnb_apply(const float* __restrict__ x, const float* __restrict__ dxo,
                                                   const float* __restrict__ gamma, const float* __restrict__ stats,
                                                   const double* __restrict__ sums, long long n, int B, int act,
                                                   float* __restrict__ dx, int accumulate, float* __restrict__ dgamma,
                                                   float* __restrict__ dbeta) {
    const long long e = (long long)blockIdx.x * 256 + threadIdx.x;
    if (e >= n) return;
    const float gm = stats ? gamma[e] : 1.f;
    const float inv_n = 1.f / (float)n;
    float dg = 0.f, dbt = 0.f;
    for (int b = 0; b < B; b++) {
        const size_t i = (size_t)b * n + e;
        const float xv = x[i], d = dxo[i];
        const float lr = (!act || xv > 0.f) ? 1.f : LRELU_ALPHA;
        float g;
        if (stats) {
            const float mu = stats[2 * b], rs = stats[2 * b + 1];
            const float xh = (lrelu(xv) - mu) * rs;
            dg = fmaf(d, xh, dg);
            dbt += d;
            const float mg = (float)(sums[2 * b] * inv_n), mgh = (float)(sums[2 * b + 1] * inv_n);
            g = rs * (d * gm - mg - xh * mgh) * lr;
        } else {
            g = d * lr;
        }
        dx[i] = accumulate ? dx[i] + g : g;
    }
    if (stats) {
        dgamma[e] += dg;
        dbeta[e] += dbt;
    }
}

void launch_ln_backward(const float* x, const float* dxo, const float* gamma, const float* stats, double* sums,
                        long long n, int B, int act, float* dx, int accumulate, float* dgamma, float* dbeta,
                        hipStream_t st) {
    if (stats) hipLaunchKernelGGL(k_lnb_reduce, dim3(B), dim3(256), 0, st, x, dxo, gamma, stats, n, sums);
    hipLaunchKernelGGL(k_lnb_apply, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, x, dxo, gamma, stats, sums, n,
                       B, act, dx, accumulate, dgamma, dbeta);
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
            const float ds = g * ex * ub[e] + a.g_ld;
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
                                                  float lambda_y, float inv_batch) {
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
                     float inv_batch, hipStream_t st) {
    const long long total = (long long)B * HW * D;
    long long gx = (total + 255) / 256;
    if (gx > 8192) gx = 8192;
    hipLaunchKernelGGL(k_nll_grad, dim3((unsigned)gx), dim3(256), 0, st, xy, zy, dzy, total, D, x_d, lambda_y,
                       inv_batch);
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
