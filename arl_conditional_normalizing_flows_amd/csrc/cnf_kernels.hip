// cnf_kernels.hip — gfx950 (CDNA4) kernels of the conditional-RealNVP hot path.
//
//   k_conv      fused ResNeXt convolution: [LeakyReLU -> per-image LayerNorm (per-element
//               gamma/beta) on load] -> 1x1 or 3x3 dilated conv as an implicit GEMM on
//               v_mfma_f32_16x16x4_f32 -> [+bias, +residual] -> store -> per-tile LN-stat
//               partials (n, mean, M2) of LeakyReLU(out) for the NEXT LayerNorm.
//               (conv_cINN_base_functions.py:330-413, 501-627; conv_cINN_make_model.py:1107-1195)
//   k_gather_u1c mask compress of u into u1c (conv_cINN_make_model.py:720-759)
//   k_coupling  tanh*w, exp, affine law fwd/inv, decompress scatter, u1 copy and the per-image
//               log-det partial sum (conv_cINN_make_model.py:1198-1205, 1215-1328, 1333-1394)
//   k_ld_reduce deterministic per-image log-det reduction
//   k_map_*     squeeze/factor boundary gathers/scatters via index maps (:130-329, :1762-1770)
//   k_squeeze   space_to_depth / depth_to_space in TF channel order (:179, :211)
//   k_chcopy    channel-window copy (factor split/concat, :276-327)
//   k_nll       per-image NLL terms; k_nll_sums batch sums (:1815-1848)
//
// All reductions are two-level and atomic-free (bitwise-deterministic).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <stdexcept>

#include "cnf_device.h"

namespace cnf {

// Epilogue shared by all conv kernels. Lane (i, q) of wave w holds, for subtile s = w + 4m,
// out[pixel pix0 + 16s + 4q + r][channel 16n + i] in acc[m][n][r]. Adds bias and the residual
// (ALL residual loads are issued before any store: res may alias out), stores the channels of
// the store mask, and writes the tile's LN-stat partial of LeakyReLU(out).
template <int MR, int NR>
__device__ __forceinline__ void conv_epilogue(const ConvProb& P, f4 (&acc)[MR][NR], int img, int HW, int pix0,
                                              int Pv, int tr, double* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, kq = lane >> 4;
    const int cout = P.cout;
    float* __restrict__ out = P.out;
    const float* res = P.res;
    bool chv[NR], st[NR];
    float bias[NR];
#pragma unroll
    for (int n = 0; n < NR; n++) {
        const int ch = n * 16 + i16;
        chv[n] = ch < cout;
        bias[n] = chv[n] ? P.bias[ch] : 0.f;
        st[n] = chv[n] && stored(P, ch);
    }
    size_t oe[MR][4];
    bool pv[MR][4];
#pragma unroll
    for (int m = 0; m < MR; m++)
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const int p = (wave + 4 * m) * 16 + kq * 4 + r;
            pv[m][r] = p < Pv;
            oe[m][r] = ((size_t)img * HW + pix0 + (pv[m][r] ? p : 0)) * P.out_cs + P.out_off;
        }
    if (res != nullptr) {
        float rv[MR][NR][4];
#pragma unroll
        for (int m = 0; m < MR; m++)
#pragma unroll
            for (int n = 0; n < NR; n++)
#pragma unroll
                for (int r = 0; r < 4; r++) rv[m][n][r] = res[oe[m][r] + (chv[n] ? n * 16 + i16 : 0)];
#pragma unroll
        for (int m = 0; m < MR; m++)
#pragma unroll
            for (int n = 0; n < NR; n++)
#pragma unroll
                for (int r = 0; r < 4; r++) acc[m][n][r] += rv[m][n][r];
    }
#pragma unroll
    for (int m = 0; m < MR; m++)
#pragma unroll
        for (int n = 0; n < NR; n++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                acc[m][n][r] += bias[n];
                if (pv[m][r] && st[n]) out[oe[m][r] + n * 16 + i16] = acc[m][n][r];
            }
    if (P.out_part != nullptr) {
        float vals[MR * NR * 4];
        bool valid[MR * NR * 4];
#pragma unroll
        for (int m = 0; m < MR; m++)
#pragma unroll
            for (int n = 0; n < NR; n++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    vals[(m * NR + n) * 4 + r] = lrelu(acc[m][n][r]);
                    valid[(m * NR + n) * 4 + r] = pv[m][r] && chv[n];
                }
        ln_partial(vals, valid,
                   P.out_part + ((size_t)img * P.part_stride + P.out_part_base + tr * 4 + (threadIdx.x >> 6)) * LNP);
    }
}

// Register-streamed GEMM over the run of `npx` pixels starting at pixel p0 of image img:
// acc[m][n] += A * B with A[p][c] = LN(LeakyReLU(in[p][c])) loaded as float4 per lane (K
// permuted: lane (i, q) holds channels 16g + 4q + s at k-step s of channel group g) and B from
// the LDS image lw ([g][q][j][s]). Wave w owns 16-pixel subtiles w, w+4, ... Branch-free MFMA
// loop; pixels/channels beyond the valid range feed zeros.
template <int MR, int NR, bool VEC>
__device__ __forceinline__ void gemm_stream(const ConvProb& P, int img, int HW, int p0, int npx, const float* lw,
                                            int G, float mu, float rstd, bool has_ln, f4 (&acc)[MR][NR]) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, kq = lane >> 4;
    const int cin = P.cin;
    const bool act = P.act != 0;
    constexpr int NSJ = 16 * NR;
    bool pval[MR];
    size_t xoff[MR];
#pragma unroll
    for (int m = 0; m < MR; m++) {
        const int p = (wave + 4 * m) * 16 + i16;
        pval[m] = p < npx;
        xoff[m] = (size_t)(p0 + (pval[m] ? p : 0)) * P.in_cs + P.in_off;
    }
    const float* __restrict__ xb = P.in + (size_t)img * HW * P.in_cs;
    const float* __restrict__ gp = P.gamma;
    const float* __restrict__ bp = P.beta;
#pragma unroll
    for (int m = 0; m < MR; m++)
#pragma unroll
        for (int n = 0; n < NR; n++) acc[m][n] = f4{0.f, 0.f, 0.f, 0.f};

    auto load_group = [&](int g, f4 (&xr)[MR], f4 (&gr)[MR], f4 (&br)[MR]) {
        const int c0 = 16 * g + 4 * kq;
#pragma unroll
        for (int m = 0; m < MR; m++) {
            if (VEC) {
                const size_t e = xoff[m] + (c0 < cin ? c0 : 0);
                xr[m] = *reinterpret_cast<const f4*>(xb + e);
                if (has_ln) {
                    gr[m] = *reinterpret_cast<const f4*>(gp + e);
                    br[m] = *reinterpret_cast<const f4*>(bp + e);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const size_t e = xoff[m] + (c0 + j < cin ? c0 + j : 0);
                    xr[m][j] = xb[e];
                    if (has_ln) {
                        gr[m][j] = gp[e];
                        br[m][j] = bp[e];
                    }
                }
            }
        }
    };

    f4 xr[MR], gr[MR], br[MR];
#pragma unroll
    for (int m = 0; m < MR; m++) {
        xr[m] = f4{0.f, 0.f, 0.f, 0.f};
        gr[m] = f4{1.f, 1.f, 1.f, 1.f};
        br[m] = f4{0.f, 0.f, 0.f, 0.f};
    }
    load_group(0, xr, gr, br);
    for (int g = 0; g < G; g++) {
        f4 xn[MR], gn[MR], bn[MR];
#pragma unroll
        for (int m = 0; m < MR; m++) {
            gn[m] = gr[m];
            bn[m] = br[m];
            xn[m] = xr[m];
        }
        if (g + 1 < G) load_group(g + 1, xn, gn, bn);
        const int c0 = 16 * g + 4 * kq;
        float av[MR][4];
#pragma unroll
        for (int m = 0; m < MR; m++)
#pragma unroll
            for (int j = 0; j < 4; j++) {
                float x = xr[m][j];
                if (act) x = lrelu(x);
                if (has_ln) x = (x - mu) * rstd * gr[m][j] + br[m][j];
                av[m][j] = (pval[m] && c0 + j < cin) ? x : 0.f;
            }
        f4 bq[NR];
        const float* brow = lw + ((size_t)(g * 4 + kq) * NSJ + i16) * 4;
#pragma unroll
        for (int n = 0; n < NR; n++) bq[n] = *reinterpret_cast<const f4*>(brow + n * 64);
#pragma unroll
        for (int s = 0; s < 4; s++)
#pragma unroll
            for (int m = 0; m < MR; m++)
#pragma unroll
                for (int n = 0; n < NR; n++)
                    acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m][s], bq[n][s], acc[m][n], 0, 0, 0);
#pragma unroll
        for (int m = 0; m < MR; m++) {
            xr[m] = xn[m];
            gr[m] = gn[m];
            br[m] = bn[m];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// k_conv1: 1x1 convolution (conv_a / conv_b of dilated_residual_block,
// conv_cINN_base_functions.py:561-565, 609-613) with the A operand streamed from HBM straight
// into registers (gemm_stream) and LN-on-load; tiles are runs of P pixels inside one image.
// ---------------------------------------------------------------------------------------------
template <int MR, int NR, bool VEC>
__device__ __forceinline__ void conv1_body(const ConvArgs& a, const ConvProb& P, unsigned char* smem) {
    const int HW = a.H * a.W;
    const int img = blockIdx.x / a.tiles_per_img;
    const int tr = blockIdx.x - img * a.tiles_per_img;
    const int px0 = tr * a.P;
    const int Pv = min(a.P, HW - px0);
    const int G = (P.cin + 15) >> 4;
    double* red = reinterpret_cast<double*>(smem);
    float* lw = reinterpret_cast<float*>(smem + P.lds_w_off);
    float mu, rstd;
    in_ln(P, img, mu, rstd);
    copy_to_lds<256>(P.wt, lw, G * 16 * 16 * NR);   // pre-packed B image (PK_1X1)
    __syncthreads();
    const bool has_ln = P.in_part != nullptr;
    f4 acc[MR][NR];
    gemm_stream<MR, NR, VEC>(P, img, HW, px0, Pv, lw, G, mu, rstd, has_ln, acc);
    conv_epilogue<MR, NR>(P, acc, img, HW, px0, Pv, tr, red);
}

template <int MR, bool VEC, int ROLE>
__global__ __launch_bounds__(256) void k_conv1(ConvArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const ConvProb P = a.p[blockIdx.y];
    switch (P.nr) {
        case 1: conv1_body<MR, 1, VEC>(a, P, smem); break;
        case 2: conv1_body<MR, 2, VEC>(a, P, smem); break;
        case 3: conv1_body<MR, 3, VEC>(a, P, smem); break;
        default: conv1_body<MR, 4, VEC>(a, P, smem); break;
    }
}

// ---------------------------------------------------------------------------------------------
// k_conv: 3x3 dilated convolution as an implicit GEMM from an LDS-staged, normalised input band
// (conv_in :1114-1119, the grouped dilated branches conv_cINN_base_functions.py:389-411, and
// conv_out when cout > 7). Tile = TH image rows; the band (+d halo rows/cols, zero padded) is
// staged once; A[p][k=(tap,c)] = lin[abase(p) + koff(k)], B[k][n] from LDS.
// ---------------------------------------------------------------------------------------------
template <int MR, int NR>
__device__ __forceinline__ void conv3_body(const ConvArgs& a, const ConvProb& P, unsigned char* smem) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int img = blockIdx.x / a.tiles_per_img;
    const int tr = blockIdx.x - img * a.tiles_per_img;
    const int H = a.H, W = a.W, TH = a.TH;
    const int HW = H * W;
    const int r0 = tr * TH;
    const int rows = min(TH, H - r0);
    const int Pv = rows * W;      // valid output pixels of this tile
    const int PT = TH * W;        // staged (padded) pixels
    const int d = P.dil;
    const int WP = W + 2 * d;
    const int S = P.S, cin = P.cin, K = 9 * cin, Kpad = P.Kpad, NS = P.NS, cout = P.cout;
    double* red = reinterpret_cast<double*>(smem);
    float* lin = reinterpret_cast<float*>(smem + P.lds_in_off);
    float* lw = reinterpret_cast<float*>(smem + P.lds_w_off);
    int* lk = reinterpret_cast<int*>(smem + P.lds_k_off);

    float mu, rstd;
    in_ln(P, img, mu, rstd);
    copy_to_lds<256>(P.wt, lw, Kpad * NS);   // pre-packed [Kpad][NS] (PK_KN)
    // per-k LDS offsets of the A operand (tap, channel)
    for (int k = tid; k < Kpad; k += 256) {
        int off = 0;
        if (k < K) {
            const int tap = k / cin, ci = k - tap * cin;
            const int kh = tap / 3, kw = tap - kh * 3;
            off = (kh * d * WP + kw * d) * S + ci;
        }
        lk[k] = off;
    }
    __syncthreads();
    const bool has_ln = P.in_part != nullptr;
    // stage the (normalised) input band (+halo) into LDS; magic-number divisions, batched loads
    {
        const float* __restrict__ inb = P.in + (size_t)img * HW * P.in_cs + P.in_off;
        const float* __restrict__ gb = has_ln ? P.gamma + P.in_off : nullptr;
        const float* __restrict__ bb = has_ln ? P.beta + P.in_off : nullptr;
        const bool act = P.act != 0;
        const int SR = TH + 2 * d;
        const int total = SR * WP * cin;
        const uint32_t cmag = P.cin_mag, wmag = P.wp_mag;
        const int in_cs = P.in_cs;
        for (int base = 0; base < total; base += 256 * 4) {
            float xv[4], gv[4], bv[4];
            int li[4];
            bool ok[4];
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int idx = base + u * 256 + tid;
                const int pix = (cin == 1) ? idx : (int)__umulhi((uint32_t)idx, cmag);
                const int c = idx - pix * cin;
                const int rr = (int)__umulhi((uint32_t)pix, wmag);
                const int cc = pix - rr * WP;
                const int row = r0 - d + rr, col = cc - d;
                li[u] = (idx < total) ? pix * S + c : -1;
                ok[u] = idx < total && row >= 0 && row < H && col >= 0 && col < W;
                const size_t e = ok[u] ? (size_t)(row * W + col) * in_cs + c : 0;
                xv[u] = inb[e];
                if (has_ln) {
                    gv[u] = gb[e];
                    bv[u] = bb[e];
                }
            }
#pragma unroll
            for (int u = 0; u < 4; u++) {
                if (li[u] < 0) continue;
                float x = xv[u];
                if (act) x = lrelu(x);
                if (has_ln) x = (x - mu) * rstd * gv[u] + bv[u];
                lin[li[u]] = ok[u] ? x : 0.f;
            }
        }
    }
    __syncthreads();

    const int i16 = lane & 15, kq = lane >> 4;
    int abase[MR];
#pragma unroll
    for (int m = 0; m < MR; m++) {
        int p = (wave + 4 * m) * 16 + i16;
        if (p >= PT) p = 0;
        const int pr = p / W, pc = p - pr * W;
        abase[m] = (pr * WP + pc) * S;
    }
    f4 acc[MR][NR];
#pragma unroll
    for (int m = 0; m < MR; m++)
#pragma unroll
        for (int n = 0; n < NR; n++) acc[m][n] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 4
    for (int k0 = 0; k0 < Kpad; k0 += 4) {
        const int kr = k0 + kq;
        const int ko = lk[kr];
        const float* wrow = lw + kr * NS + i16;
        float bv[NR];
#pragma unroll
        for (int n = 0; n < NR; n++) bv[n] = wrow[n * 16];
#pragma unroll
        for (int m = 0; m < MR; m++) {
            const float av = lin[abase[m] + ko];
#pragma unroll
            for (int n = 0; n < NR; n++)
                acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, bv[n], acc[m][n], 0, 0, 0);
        }
    }
    conv_epilogue<MR, NR>(P, acc, img, HW, r0 * W, Pv, tr, red);
}

template <int KS, int MR, int ROLE>
__global__ __launch_bounds__(256) void k_conv(ConvArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const ConvProb P = a.p[blockIdx.y];
    switch (P.nr) {
        case 1: conv3_body<MR, 1>(a, P, smem); break;
        case 2: conv3_body<MR, 2>(a, P, smem); break;
        case 3: conv3_body<MR, 3>(a, P, smem); break;
        default: conv3_body<MR, 4>(a, P, smem); break;
    }
}

// ---------------------------------------------------------------------------------------------
// k_convtap: 3x3 (dilation 1) convolution with few output channels (conv_out, cout <= 7;
// conv_cINN_make_model.py:1150-1155, 1190-1195) as a tap-decomposed GEMM: over the halo'd band of
// rows [r0-1, r0+rows+1) compute C[p][(tap, o)] = sum_c LN(LeakyReLU(y))[p][c] * W[tap][c][o]
// (K = cin, N = 9*cout, register-streamed A), then out[p][o] = b[o] + sum_tap C[p + off(tap)][(tap, o)]
// from LDS. 3x fewer MFMAs than the implicit GEMM at cout=2 and no per-k address table.
// ---------------------------------------------------------------------------------------------
template <int MT, int NR, bool VEC>
__device__ __forceinline__ void convtap_body(const ConvArgs& a, const ConvProb& P, unsigned char* smem) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int H = a.H, W = a.W, HW = H * W, TH = a.TH;
    const int img = blockIdx.x / a.tiles_per_img;
    const int tr = blockIdx.x - img * a.tiles_per_img;
    const int r0 = tr * TH;
    const int rows = min(TH, H - r0);
    const int rb0 = max(r0 - 1, 0), rb1 = min(r0 + rows + 1, H);
    const int nband = (rb1 - rb0) * W;
    const int cin = P.cin, cout = P.cout;
    const int G = (cin + 15) >> 4;
    constexpr int NSJ = 16 * NR;
    constexpr int CS = NSJ + 1;   // LDS row stride of the C tile
    double* red = reinterpret_cast<double*>(smem);
    float* lw = reinterpret_cast<float*>(smem + P.lds_w_off);
    float* lc = reinterpret_cast<float*>(smem + P.lds_in_off);

    float mu, rstd;
    in_ln(P, img, mu, rstd);
    copy_to_lds<256>(P.wt, lw, G * 16 * NSJ);   // pre-packed tap B image (PK_TAP)
    __syncthreads();
    const bool has_ln = P.in_part != nullptr;
    f4 acc[MT][NR];
    gemm_stream<MT, NR, VEC>(P, img, HW, rb0 * W, nband, lw, G, mu, rstd, has_ln, acc);
    const int i16 = lane & 15, kq = lane >> 4;
#pragma unroll
    for (int m = 0; m < MT; m++)
#pragma unroll
        for (int n = 0; n < NR; n++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int p = (wave + 4 * m) * 16 + kq * 4 + r;
                if (p < nband) lc[p * CS + n * 16 + i16] = acc[m][n][r];
            }
    __syncthreads();
    const int nout = rows * W * cout;
    float* __restrict__ out = P.out;
    for (int e = tid; e < nout; e += 256) {
        const int p = e / cout, o = e - p * cout;
        const int pr = p / W, pc = p - pr * W;
        const int row = r0 + pr;
        float s1 = P.bias[o];
#pragma unroll
        for (int kh = 0; kh < 3; kh++) {
            const int sr = row + kh - 1;
            if (sr < 0 || sr >= H) continue;
#pragma unroll
            for (int kw = 0; kw < 3; kw++) {
                const int sc = pc + kw - 1;
                if (sc < 0 || sc >= W) continue;
                s1 += lc[((sr - rb0) * W + sc) * CS + (kh * 3 + kw) * cout + o];
            }
        }
        out[((size_t)img * HW + (size_t)row * W + pc) * P.out_cs + P.out_off + o] = s1;
    }
}

template <int MT, bool VEC>
__global__ __launch_bounds__(256) void k_convtap(ConvArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const ConvProb P = a.p[blockIdx.y];
    switch (P.nr) {
        case 1: convtap_body<MT, 1, VEC>(a, P, smem); break;
        case 2: convtap_body<MT, 2, VEC>(a, P, smem); break;
        case 3: convtap_body<MT, 3, VEC>(a, P, smem); break;
        default: convtap_body<MT, 4, VEC>(a, P, smem); break;
    }
}

// ---------------------------------------------------------------------------------------------
// masks (conv_cINN_make_model.py:720-759, 896-1071)
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gather_u1c(const float* __restrict__ u, float* __restrict__ u1c, int H,
                                                    int W, int D, int mask, int hc, int wc, int dc1) {
    const int img = blockIdx.y;
    const int n = hc * wc * dc1;
    const float* ub = u + (size_t)img * H * W * D;
    float* ob = u1c + (size_t)img * n;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < n; e += gridDim.x * 256) {
        const int p = e / dc1, c = e - p * dc1;
        ob[e] = ub[mask_pos(mask, p, c, wc, W, D)];
    }
}

// u -> v: copy the mask half, apply the affine law to the complement half.
// dir=+1: v2 = exp(s)*u2 + t ; dir=-1: u2 = (1/exp(s)) * (v2 - t). s = w * tanh(s_pre).
__global__ __launch_bounds__(256) void k_coupling(CoupArgs a) {
    const int img = blockIdx.y;
    const int HWD = a.H * a.W * a.D;
    const int npx = a.hc * a.wc;
    const float* __restrict__ ub = a.u + (size_t)img * HWD;
    float* __restrict__ vb = a.v + (size_t)img * HWD;
    const float* __restrict__ sb = a.s_pre + (size_t)img * npx * a.dc2;
    const float* __restrict__ tb = a.t + (size_t)img * npx * a.dc2;
    const float w = *a.tanh_w;
    float lsum = 0.f;
    // one thread per element: the transformed half (coalesced s, t reads) first, then the copy of
    // the conditioning half (small layers have few pixels but many channels per pixel)
    const int n2 = npx * a.dc2, n1 = npx * a.dc1;
    for (int e = blockIdx.x * 256 + threadIdx.x; e < n2 + n1; e += gridDim.x * 256) {
        if (e < n2) {
            const int p = e / a.dc2, c = e - p * a.dc2;
            const int q = mask_pos(a.mask_c, p, c, a.wc, a.W, a.D);
            float sp, t;
            if (a.tc[0] != nullptr) {
                // out[p][c] = b[c] + sum_tap C[p + off(tap)][(tap, c)], taps in (kh, kw) order
                const int pr = p / a.wc, pc = p - pr * a.wc;
                const int ncol = 9 * a.dc2;
                const float* c0 = a.tc[0] + (size_t)img * npx * ncol;
                const float* c1 = a.tc[1] + (size_t)img * npx * ncol;
                sp = a.tbias[0][c];
                t = a.tbias[1][c];
#pragma unroll
                for (int kh = 0; kh < 3; kh++) {
                    const int sr = pr + kh - 1;
                    if (sr < 0 || sr >= a.hc) continue;
#pragma unroll
                    for (int kw = 0; kw < 3; kw++) {
                        const int sc = pc + kw - 1;
                        if (sc < 0 || sc >= a.wc) continue;
                        const size_t ci = (size_t)(sr * a.wc + sc) * ncol + (kh * 3 + kw) * a.dc2 + c;
                        sp += c0[ci];
                        t += c1[ci];
                    }
                }
                a.so_w[0][(size_t)img * npx * a.dc2 + e] = sp;
                a.so_w[1][(size_t)img * npx * a.dc2 + e] = t;
            } else {
                sp = sb[e];
                t = tb[e];
            }
            const float s = w * cpl_tanh(sp);
            vb[q] = cpl_law(s, ub[q], t, a.dir);   // (k_net_lds / k_map2 apply a deferred coupling with the same expression)
            if (a.dir > 0) lsum += s;
        } else {
            const int e1 = e - n2;
            const int p = e1 / a.dc1, c = e1 - p * a.dc1;
            const int q = mask_pos(a.mask, p, c, a.wc, a.W, a.D);
            vb[q] = ub[q];
        }
    }
    if (a.ld_part != nullptr) {
        __shared__ double sred[4];
        double ws = wave_sum((double)lsum);
        if ((threadIdx.x & 63) == 0) sred[threadIdx.x >> 6] = ws;
        __syncthreads();
        if (threadIdx.x == 0)
            a.ld_part[(size_t)img * gridDim.x + blockIdx.x] = sred[0] + sred[1] + sred[2] + sred[3];
    }
}

// Merge of one tensor's per-wave LN partial slots into slot 0 (in place), for tensors of the large
// streamed layers whose producers write more slots per image than a consumer wave folds in one pass
// (> 64): every consumer workgroup would otherwise re-read all of them for each of its images.
// One workgroup per (image, net): each thread folds its strided slots (Chan merge, as ln_fold), the
// waves merge their lanes in the parallel-axis form, thread 0 the four waves in order; the result is
// stored as the single slot (mean, 0, M2, N), which ln_fold reads back as exactly that (mean, M2, N).
// Fixed order throughout: deterministic.
__global__ __launch_bounds__(256) void k_ln_merge(float* __restrict__ part0, float* __restrict__ part1, int nparts,
                                                   int part_stride) {
    const int img = blockIdx.x;
    float* q = (blockIdx.y == 0 ? part0 : part1) + (size_t)img * part_stride * LNP;
    float n = 0.f, m = 0.f, M2 = 0.f;
    for (int i0 = threadIdx.x; i0 < nparts; i0 += 4 * 256) {
        f4 v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int i = i0 + u * 256;
            v[u] = i < nparts ? *reinterpret_cast<const f4*>(q + (size_t)LNP * i) : f4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < 4; u++) ln_fold(v[u], n, m, M2);
    }
    // wave: N = sum n, mean = sum n m / N, M2 = sum (M2 + n (m - mean)^2)
    const float N = wave_sum_f(n);
    const float mean = N > 0.f ? wave_sum_f(n * m) / N : 0.f;
    const float d = m - mean;
    const float M = wave_sum_f(fmaf(n * d, d, M2));
    __shared__ float wv[4][3];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    if (lane == 0) {
        wv[wave][0] = N;
        wv[wave][1] = mean;
        wv[wave][2] = M;
    }
    __syncthreads();   // every slot has been read: slot 0 may be overwritten
    if (threadIdx.x == 0) {
        float tn = 0.f, tm = 0.f, tM = 0.f;
        for (int w = 0; w < 4; w++) {
            const float wn = wv[w][0];
            if (wn > 0.f) {
                const float nn = tn + wn, dl = wv[w][1] - tm, f = wn / nn;
                tm = fmaf(dl, f, tm);
                tM = tM + wv[w][2] + dl * dl * tn * f;
                tn = nn;
            }
        }
        *reinterpret_cast<f4*>(q) = f4{tm, 0.f, tM, tn};
    }
}

// out[img] (=|+=) sum over nl layers, np parts of part[((l*B)+img)*np + j]: one wave per image,
// lane k folds entries k, k+64, ... (all its loads in flight together), then a fixed-order wave sum
__global__ __launch_bounds__(64) void k_ld_reduce(const double* __restrict__ part, float* __restrict__ out, int B,
                                                  int nl, int np, int accumulate) {
    const int img = blockIdx.x, lane = threadIdx.x;
    const int n = nl * np;
    double s = 0.0;
    for (int k0 = 0; k0 < n; k0 += 256) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int k = k0 + 64 * u + lane;
            const int l = k / np, j = k - l * np;
            v[u] = k < n ? part[((size_t)l * B + img) * np + j] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) s += v[u];
    }
    s = wave_sum(s);
    if (lane == 0) out[img] = accumulate ? (float)((double)out[img] + s) : (float)s;
}

// dst[b, i] = src[b, idx[i]]
__global__ __launch_bounds__(256) void k_map_gather(const float* __restrict__ src, float* __restrict__ dst,
                                                    const int* __restrict__ idx, int n, int src_stride,
                                                    int dst_stride) {
    const int img = blockIdx.y;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256)
        dst[(size_t)img * dst_stride + i] = src[(size_t)img * src_stride + idx[i]];
}

// dst[b, idx[i]] = src[b, sidx ? sidx[i] : i]
__global__ __launch_bounds__(256) void k_map_scatter(const float* __restrict__ src, float* __restrict__ dst,
                                                     const int* __restrict__ sidx, const int* __restrict__ didx,
                                                     int n, int src_stride, int dst_stride) {
    const int img = blockIdx.y;
    for (int i = blockIdx.x * 256 + threadIdx.x; i < n; i += gridDim.x * 256) {
        int s = sidx ? sidx[i] : i;
        dst[(size_t)img * dst_stride + didx[i]] = src[(size_t)img * src_stride + s];
    }
}

// blocks [0, ga): map a; [ga, ga + gb): map b (each reading its source through the pending coupling
// when MapOp::pend); block ga + gb (when r.part, or a pending forward coupling): the log-det work of
// image blockIdx.y by wave 0 — layer k's sum of s for a pending forward coupling, and / or the
// reduction of the partial slots (as k_ld_reduce)
__global__ __launch_bounds__(256) void k_map2(MapOp a, MapOp b, int ga, int gb, LdReduce r, CoupPend q, int B) {
    const int img = blockIdx.y;
    const int bx = blockIdx.x;
    const int n_img = q.on ? q.hc * q.wc * (q.dc1 + q.dc2) : 0;   // elements of u_k per image
    if (bx < ga + gb) {
        const MapOp& m = bx < ga ? a : b;
        const int g0 = bx < ga ? 0 : ga, gn = bx < ga ? ga : gb;
        if (q.on && m.pend) {
            const float* ub = q.u + (size_t)img * n_img;
            const size_t sb = (size_t)img * q.hc * q.wc * q.dc2;
            const float w = *q.tanh_w;
            for (int i = (bx - g0) * 256 + threadIdx.x; i < m.n; i += gn * 256) {
                const int s = m.sidx ? m.sidx[i] : i;
                const int d = m.didx ? m.didx[i] : i;
                const int ci = pend_index(q, s, q.W, q.D);
                float v = ub[s];
                if (ci >= 0) v = cpl_law(w * cpl_tanh(q.s_pre[sb + ci]), v, q.t[sb + ci], q.dir);   // k_coupling's expression
                m.dst[(size_t)img * m.ds + d] = v;
            }
        } else {
            for (int i = (bx - g0) * 256 + threadIdx.x; i < m.n; i += gn * 256) {
                const int s = m.sidx ? m.sidx[i] : i;
                const int d = m.didx ? m.didx[i] : i;
                m.dst[(size_t)img * m.ds + d] = m.src[(size_t)img * m.ss + s];
            }
        }
        return;
    }
    if (threadIdx.x >= 64) return;
    const int lane = threadIdx.x;
    double acc = 0.0;
    if (q.on && q.ld_part != nullptr) {
        const int n2 = q.hc * q.wc * q.dc2;
        const float* sp = q.s_pre + (size_t)img * n2;
        const float w = *q.tanh_w;
        float ls = 0.f;
        for (int e = lane; e < n2; e += 64) ls += w * cpl_tanh(sp[e]);
        const double t = wave_sum((double)ls);
        if (r.part == nullptr) {
            if (lane < q.np) q.ld_part[(size_t)img * q.np + lane] = lane == 0 ? t : 0.0;
            return;
        }
        acc = t;
    }
    const int n = r.nl * r.np;
    double ps = 0.0;
    for (int k0 = 0; k0 < n; k0 += 256) {
        double v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int k = k0 + 64 * u + lane;
            const int l = k / r.np, j = k - l * r.np;
            v[u] = k < n ? r.part[((size_t)l * B + img) * r.np + j] : 0.0;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) ps += v[u];
    }
    acc += wave_sum(ps);
    if (lane == 0) r.out[img] = r.accumulate ? (float)((double)r.out[img] + acc) : (float)acc;
}

// dir=+1: out[b,i,j,(di*2+dj)*C+c] = in[b,2i+di,2j+dj,c] (in: H x W x C)
// dir=-1: inverse (in: H x W x 4C', out 2H x 2W x C')
__global__ __launch_bounds__(256) void k_squeeze(const float* __restrict__ in, float* __restrict__ out, int H,
                                                 int W, int C, int dir, long long total) {
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        if (dir > 0) {
            // e indexes out: (b, i, j, q) with q in [0, 4C)
            const int C4 = 4 * C, H2 = H / 2, W2 = W / 2;
            long long t = e;
            int q = (int)(t % C4);
            t /= C4;
            int j = (int)(t % W2);
            t /= W2;
            int i = (int)(t % H2);
            long long b = t / H2;
            int blk = q / C, c = q - blk * C;
            int di = blk >> 1, dj = blk & 1;
            out[e] = in[((b * H + 2 * i + di) * W + 2 * j + dj) * C + c];
        } else {
            // e indexes out (b, y, x, c) of shape 2H x 2W x C'  with C' = C/4
            const int Cp = C / 4, H2 = 2 * H, W2 = 2 * W;
            long long t = e;
            int c = (int)(t % Cp);
            t /= Cp;
            int x = (int)(t % W2);
            t /= W2;
            int y = (int)(t % H2);
            long long b = t / H2;
            int i = y >> 1, di = y & 1, j = x >> 1, dj = x & 1;
            out[e] = in[((b * H + i) * W + j) * C + (di * 2 + dj) * Cp + c];
        }
    }
}

__global__ __launch_bounds__(256) void k_chcopy(const float* __restrict__ in, int in_cs, int in_off,
                                                float* __restrict__ out, int out_cs, int out_off, int C,
                                                long long npix) {
    const long long total = npix * C;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < total; e += (long long)gridDim.x * 256) {
        long long p = e / C;
        int c = (int)(e - p * C);
        out[p * out_cs + out_off + c] = in[p * in_cs + in_off + c];
    }
}

// the four batch sums of the per-image terms, in image order (one wave): shared by k_nll's last
// workgroup and the standalone k_nll_sums of the toy path
__device__ __forceinline__ void nll_batch_sums(const float* per_image, float* sums, int B, int lane) {
    double a = 0, bz = 0, by = 0, bl = 0;
    for (int i = lane; i < B; i += 64) {
        double llz = per_image[i * 3], lly = per_image[i * 3 + 1], ld = per_image[i * 3 + 2];
        a += -(llz + lly + ld);
        bz += -llz;
        by += -lly;
        bl += -ld;
    }
    a = wave_sum(a);
    bz = wave_sum(bz);
    by = wave_sum(by);
    bl = wave_sum(bl);
    if (lane == 0) {
        sums[0] = (float)a;
        sums[1] = (float)bz;
        sums[2] = (float)by;
        sums[3] = (float)bl;
    }
}

__global__ void k_nll_sums(const float* __restrict__ per_image, float* __restrict__ sums, int B) {
    nll_batch_sums(per_image, sums, B, threadIdx.x);   // 64 threads
}

// per-image NLL terms: llz = sum_{h,w} (-0.5|z|^2 - x_d/2 ln 2pi), lly = -lambda*sum|y-y'|, ld
__global__ __launch_bounds__(256) void k_nll(const float* __restrict__ xy, const float* __restrict__ zy,
                                             const float* __restrict__ ld, float* __restrict__ per_image,
                                             float* __restrict__ sums, unsigned* __restrict__ done, int HW,
                                             int D, int x_d, float lambda_y) {
    const int img = blockIdx.x;
    const float* xb = xy + (size_t)img * HW * D;
    const float* zb = zy + (size_t)img * HW * D;
    const int n = HW * D;
    double zz = 0.0, ya = 0.0;
    // 8 elements per thread and pass, every load issued before the first use
    for (int e0 = threadIdx.x; e0 < n; e0 += 8 * 256) {
        float z[8], x[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int e = e0 + 256 * u;
            z[u] = e < n ? zb[e] : 0.f;
            x[u] = e < n && e % D >= x_d ? xb[e] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int e = e0 + 256 * u;
            if (e >= n) continue;
            if (e % D < x_d)
                zz += (double)(z[u] * z[u]);
            else
                ya += (double)fabsf(z[u] - x[u]);
        }
    }
    __shared__ double s1[4], s2[4];
    double a = wave_sum(zz), b = wave_sum(ya);
    if ((threadIdx.x & 63) == 0) {
        s1[threadIdx.x >> 6] = a;
        s2[threadIdx.x >> 6] = b;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        double z2 = s1[0] + s1[1] + s1[2] + s1[3];
        double ay = s2[0] + s2[1] + s2[2] + s2[3];
        double llz = -0.5 * z2 - 0.5 * (double)x_d * LOG_2PI_D * (double)HW;
        double lly = -(double)lambda_y * ay;
        per_image[img * 3 + 0] = (float)llz;
        per_image[img * 3 + 1] = (float)lly;
        per_image[img * 3 + 2] = ld[img];
    }
    // the batch sums in the same launch: the workgroup that finishes last (the wrapping counter
    // reads B - 1 and returns to 0 for the next call) adds the per-image terms in image order, so
    // the result does not depend on which workgroup that is. The agent-scope fences publish every
    // workgroup's terms across the XCDs' L2s before the counter moves, and the last one's loads
    // after it.
    __shared__ int last;
    if (threadIdx.x == 0) {
        __threadfence();
        last = atomicInc(done, (unsigned)gridDim.x - 1u) == gridDim.x - 1u;
    }
    __syncthreads();
    if (last && threadIdx.x < 64) {
        __threadfence();
        nll_batch_sums(per_image, sums, gridDim.x, threadIdx.x);
    }
}


// aux[i] = map[i] >= 0 ? params[map[i]] : 0
__global__ __launch_bounds__(256) void k_pack(const float* __restrict__ params, const int64_t* __restrict__ map,
                                              float* __restrict__ aux, long long n) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        int64_t s = map[i];
        aux[i] = s >= 0 ? params[s] : 0.f;
    }
}

void launch_conv(int ks, int mr, int role, const ConvArgs& a, int grid_x, int lds, hipStream_t st) {
    dim3 g(grid_x, a.nprob), b(256);
#define CNF_CONV_CASE(MR_, R_) \
    if (ks == 3 && mr == MR_ && role == R_) { CNF_LAUNCH((k_conv<3, MR_, R_>), g, b, lds, st, a); return; }
    CNF_CONV_CASE(1, ROLE_CONV_IN)
    CNF_CONV_CASE(1, ROLE_GC)
    CNF_CONV_CASE(1, ROLE_CONV_OUT)
    CNF_CONV_CASE(2, ROLE_CONV_IN)
    CNF_CONV_CASE(2, ROLE_GC)
    CNF_CONV_CASE(2, ROLE_CONV_OUT)
#undef CNF_CONV_CASE
}

void launch_conv1(int mr, bool vec, int role, const ConvArgs& a, int grid_x, int lds, hipStream_t st) {
    dim3 g(grid_x, a.nprob), b(256);
#define CNF_CONV1_CASE(MR_, V_, R_) \
    if (mr == MR_ && vec == V_ && role == R_) { CNF_LAUNCH((k_conv1<MR_, V_, R_>), g, b, lds, st, a); return; }
    CNF_CONV1_CASE(1, true, ROLE_CONV_A)
    CNF_CONV1_CASE(1, true, ROLE_CONV_B)
    CNF_CONV1_CASE(1, false, ROLE_CONV_A)
    CNF_CONV1_CASE(1, false, ROLE_CONV_B)
    CNF_CONV1_CASE(2, true, ROLE_CONV_A)
    CNF_CONV1_CASE(2, true, ROLE_CONV_B)
    CNF_CONV1_CASE(2, false, ROLE_CONV_A)
    CNF_CONV1_CASE(2, false, ROLE_CONV_B)
#undef CNF_CONV1_CASE
}

void launch_convtap(int mt, bool vec, const ConvArgs& a, int grid_x, int lds, hipStream_t st) {
    dim3 g(grid_x, a.nprob), b(256);
#define CNF_TAP_CASE(MT_, V_) \
    if (mt == MT_ && vec == V_) { CNF_LAUNCH((k_convtap<MT_, V_>), g, b, lds, st, a); return; }
    CNF_TAP_CASE(1, true) CNF_TAP_CASE(2, true) CNF_TAP_CASE(3, true) CNF_TAP_CASE(4, true) CNF_TAP_CASE(6, true)
    CNF_TAP_CASE(1, false) CNF_TAP_CASE(2, false) CNF_TAP_CASE(3, false) CNF_TAP_CASE(4, false) CNF_TAP_CASE(6, false)
#undef CNF_TAP_CASE
}

void launch_gather_u1c(const float* u, float* u1c, int B, int H, int W, int D, int mask, int hc, int wc, int dc1,
                       hipStream_t st) {
    int n = hc * wc * dc1;
    int gx = (n + 255) / 256;
    if (gx > 64) gx = 64;
    CNF_LAUNCH(k_gather_u1c, dim3(gx, B), dim3(256), 0, st, u, u1c, H, W, D, mask, hc, wc, dc1);
}

void launch_coupling(const CoupArgs& a, int B, int nparts, hipStream_t st) {
    CNF_LAUNCH(k_coupling, dim3(nparts, B), dim3(256), 0, st, a);
}

// Training forward of a streamed layer: (mean, rstd) of one LN tensor per (image, net) from its
// producer's partial slots, folded exactly as the consumer kernels fold them (in_ln): the statistics
// the backward uses are bitwise the forward's. One wave per (image, net).
__global__ __launch_bounds__(64) void k_ln_final(LnFinalSet a) {
    const int img = blockIdx.x, t = blockIdx.y >> 1, net = blockIdx.y & 1, lane = threadIdx.x;
    const float* q = a.part[t][net] + (size_t)img * a.part_stride * LNP;
    const int nparts = a.nparts[t];
    // the lane's slots lane, lane + 64, ... folded in in_ln_finish's order (the first one by
    // ln_fold_first), so (mu, rstd) are the consumer kernels' bits
    float n, m, M2;
    ln_fold_first(lane < nparts ? *reinterpret_cast<const f4*>(q + (size_t)LNP * lane) : f4{0.f, 0.f, 0.f, 0.f}, n, m, M2);
    for (int i = lane + 64; i < nparts; i += 64) ln_fold(*reinterpret_cast<const f4*>(q + (size_t)LNP * i), n, m, M2);
    float mu, rstd;
    ln_wave_final(n, m, M2, mu, rstd);
    if (lane == 0) {
        float* s = a.st[t][net];
        s[2 * img] = mu;
        s[2 * img + 1] = rstd;
    }
}

void launch_ln_final(const LnFinalSet& s, int B, hipStream_t st) {
    if (s.count <= 0) return;
    CNF_LAUNCH(k_ln_final, dim3(B, 2 * s.count), dim3(64), 0, st, s);
}

void launch_ln_merge(float* part0, float* part1, int nparts, int part_stride, int B, hipStream_t st) {
    CNF_LAUNCH(k_ln_merge, dim3(B, part1 != nullptr ? 2 : 1), dim3(256), 0, st, part0, part1, nparts, part_stride);
}

void launch_ld_reduce(const double* part, float* out, int B, int nl, int np, int accumulate, hipStream_t st) {
    CNF_LAUNCH(k_ld_reduce, dim3(B), dim3(64), 0, st, part, out, B, nl, np, accumulate);
}

void launch_map_gather(const float* src, float* dst, const int* idx, int n, int ss, int ds, int B, hipStream_t st) {
    int gx = (n + 255) / 256;
    if (gx > 64) gx = 64;
    CNF_LAUNCH(k_map_gather, dim3(gx, B), dim3(256), 0, st, src, dst, idx, n, ss, ds);
}

void launch_map_scatter(const float* src, float* dst, const int* sidx, const int* didx, int n, int ss, int ds,
                        int B, hipStream_t st) {
    int gx = (n + 255) / 256;
    if (gx > 64) gx = 64;
    CNF_LAUNCH(k_map_scatter, dim3(gx, B), dim3(256), 0, st, src, dst, sidx, didx, n, ss, ds);
}

void launch_map2(const MapOp& a, const MapOp& b, const LdReduce& r, const CoupPend& pend, int B, hipStream_t st) {
    auto gx = [](int n) { return n <= 0 ? 0 : (n + 255) / 256 > 64 ? 64 : (n + 255) / 256; };
    const int ga = gx(a.n), gb = gx(b.n);
    const int g = ga + gb + (r.part || (pend.on && pend.ld_part) ? 1 : 0);
    if (g == 0) return;
    if (pend.on && pend.np > 64) throw std::invalid_argument("k_map2: more than 64 log-det slots");
    CNF_LAUNCH(k_map2, dim3(g, B), dim3(256), 0, st, a, b, ga, gb, r, pend, B);
}

void launch_squeeze(const float* in, float* out, int B, int H, int W, int C, int dir, hipStream_t st) {
    long long total = (long long)B * H * W * C;
    long long gx = (total + 255) / 256;
    if (gx > 8192) gx = 8192;
    if (gx < 1) gx = 1;
    CNF_LAUNCH(k_squeeze, dim3((unsigned)gx), dim3(256), 0, st, in, out, H, W, C, dir, total);
}

void launch_chcopy(const float* in, int in_cs, int in_off, float* out, int out_cs, int out_off, int C, long long npix,
                   hipStream_t st) {
    long long total = npix * C;
    long long gx = (total + 255) / 256;
    if (gx > 8192) gx = 8192;
    if (gx < 1) gx = 1;
    CNF_LAUNCH(k_chcopy, dim3((unsigned)gx), dim3(256), 0, st, in, in_cs, in_off, out, out_cs, out_off, C,
                       npix);
}

void launch_nll(const float* xy, const float* zy, const float* ld, float* per_image, float* sums, unsigned* done,
                int B, int HW, int D, int x_d, float lambda_y, hipStream_t st) {
    CNF_LAUNCH(k_nll, dim3(B), dim3(256), 0, st, xy, zy, ld, per_image, sums, done, HW, D, x_d, lambda_y);
}

void launch_nll_sums(const float* per_image, float* sums, int B, hipStream_t st) {
    CNF_LAUNCH(k_nll_sums, dim3(1), dim3(64), 0, st, per_image, sums, B);
}

void launch_pack(const float* params, const int64_t* map, float* aux, long long n, hipStream_t st) {
    long long gx = (n + 255) / 256;
    if (gx > 4096) gx = 4096;
    if (gx < 1) gx = 1;
    CNF_LAUNCH(k_pack, dim3((unsigned)gx), dim3(256), 0, st, params, map, aux, n);
}

}  // namespace cnf
