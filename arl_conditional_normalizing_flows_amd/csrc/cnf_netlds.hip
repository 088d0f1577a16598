// cnf_netlds.hip — one workgroup computes a whole s,t network (net A or net b of one coupling
// layer, conv_cINN_make_model.py:1076-1213 + conv_cINN_base_functions.py:330-627) for ONE image
// with every activation resident in LDS. Used for the layers whose activations fit the 160 KiB
// LDS of a CU (the compressed images of 16x16 and below at cfg2); the per-image LayerNorm over
// H*W*C becomes an exact in-workgroup two-pass reduction and the ~11 launches of the streamed
// path collapse into one.
//
// LDS: Y (residual stream, nk ch) | T1 (nk ch) | T2 (concat of the grouped branches, gc ch;
// also the normalised input of conv_a and the gathered u1c of conv_in) | W (weights of the
// conv being run) | K (per-k tap table) | reduction scratch. Pixel strides are == 2 (mod 4) so
// the MFMA A-operand reads (16 pixels x 1 channel per 16-lane group) are bank-conflict free.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cnf_kernels.h"

namespace cnf {

typedef float f4 __attribute__((ext_vector_type(4)));

namespace {

constexpr int NW = 8;            // waves per workgroup
constexpr int NT = NW * 64;      // threads

__device__ __forceinline__ float lrelu_(float x) { return x >= 0.f ? x : LRELU_ALPHA * x; }

__device__ __forceinline__ double wsum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ double block_sum(double v, double* red) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    v = wsum(v);
    __syncthreads();
    if (lane == 0) red[wave] = v;
    __syncthreads();
    double t = 0.0;
#pragma unroll
    for (int w = 0; w < NW; w++) t += red[w];
    return t;
}

// exact two-pass per-image LN statistics of LeakyReLU(buf[p][c]) for p < HW, c < C
__device__ __forceinline__ void ln_stats(const float* buf, int stride, int HW, int C, double* red, float& mu,
                                         float& rstd) {
    const int n = HW * C;
    float s = 0.f;
    for (int e = threadIdx.x; e < n; e += NT) {
        const int p = e / C, c = e - p * C;
        s += lrelu_(buf[p * stride + c]);
    }
    const double mean = block_sum((double)s, red) / n;
    const float mf = (float)mean;
    float q = 0.f;
    for (int e = threadIdx.x; e < n; e += NT) {
        const int p = e / C, c = e - p * C;
        const float dl = lrelu_(buf[p * stride + c]) - mf;
        q += dl * dl;
    }
    double m2 = block_sum((double)q, red);
    const double dm = mean - (double)mf;
    m2 -= (double)n * dm * dm;
    if (m2 < 0.0) m2 = 0.0;
    mu = mf;
    rstd = (float)(1.0 / sqrt(m2 / n + (double)LN_EPS));
}

// dst[p][c] = LN(LeakyReLU(src[p][c])) for channels [c0, c0+nc) of a C_ln-channel LN tensor;
// gamma/beta are per (p, c) over C_ln channels (global, L2-resident). dst may alias src.
__device__ __forceinline__ void ln_apply(const float* src, int sstride, float* dst, int dstride, int HW, int c0,
                                         int nc, int C_ln, float mu, float rstd, const float* __restrict__ g,
                                         const float* __restrict__ b, bool ln) {
    const int n = HW * nc;
    for (int base = 0; base < n; base += NT * 4) {
        float xv[4], gv[4], bv[4];
        int pp[4], cc[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int e = base + u * NT + threadIdx.x;
            const int p = e / nc, c = e - p * nc;
            pp[u] = p;
            cc[u] = c;
            const bool ok = e < n;
            xv[u] = ok ? src[p * sstride + c0 + c] : 0.f;
            if (ln) {
                const size_t gi = ok ? (size_t)p * C_ln + c0 + c : 0;
                gv[u] = g[gi];
                bv[u] = b[gi];
            }
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int e = base + u * NT + threadIdx.x;
            if (e >= n) continue;
            float x = lrelu_(xv[u]);
            if (ln) x = (x - mu) * rstd * gv[u] + bv[u];
            dst[pp[u] * dstride + c0 + cc[u]] = x;
        }
    }
}

// Stage B[k][n] = wt[k*cout + n] (k < K, n < cout; zero padded to Kpad x NS) into LDS.
__device__ __forceinline__ void stage_w(const float* __restrict__ wt, int K, int cout, int Kpad, int NS, float* wl) {
    const int total = Kpad * NS;
    for (int base = 0; base < total; base += NT * 4) {
        float v[4];
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int idx = base + u * NT + threadIdx.x;
            const int k = idx / NS, n = idx - k * NS;
            v[u] = (idx < total && k < K && n < cout) ? wt[(size_t)k * cout + n] : 0.f;
        }
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int idx = base + u * NT + threadIdx.x;
            if (idx < total) wl[idx] = v[u];
        }
    }
}

__device__ __forceinline__ int ns_of(int cout) {
    int ns = (cout + 15) / 16 * 16;
    if (ns % 32 == 0) ns += 16;
    return ns;
}

// out[p][oc0 + n] = bias[n] + (res ? res[p][n] : 0) + sum_k A[p][k] B[k][n], k over
// KS*KS*cin taps x channels of `in` (LDS, channels [ic0, ic0+cin), dilation d, zero padded).
// MFMA 16x16x4 f32; each wave takes 16-pixel subtiles wave, wave+NW, ...
template <int KS, int NR>
__device__ __forceinline__ void conv_lds(const float* in, int istride, int ic0, int cin, int d, int H, int W,
                                         const float* wl, int Kpad, int NS, const int* ktab, float* out,
                                         int ostride, int oc0, int cout, const float* __restrict__ bias,
                                         bool residual) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, kq = lane >> 4;
    const int HW = H * W;
    const int nsub = (HW + 15) >> 4;
    float bz[NR];
#pragma unroll
    for (int n = 0; n < NR; n++) {
        const int ch = n * 16 + i16;
        bz[n] = ch < cout ? bias[ch] : 0.f;
    }
    for (int s = wave; s < nsub; s += NW) {
        const int p = s * 16 + i16;
        const bool pv = p < HW;
        const int pr = pv ? p / W : 0, pc = pv ? p - (p / W) * W : 0;
        f4 acc[NR];
#pragma unroll
        for (int n = 0; n < NR; n++) acc[n] = f4{0.f, 0.f, 0.f, 0.f};
        for (int k0 = 0; k0 < Kpad; k0 += 4) {
            const int k = k0 + kq;
            float av;
            if (KS == 1) {
                av = (pv && k < cin) ? in[p * istride + ic0 + k] : 0.f;
            } else {
                const int t = ktab[k];              // packed (dr+16, dc+16, c) or -1
                const int c = t & 0xffff;
                const int dr = ((t >> 24) & 0xff) - 16, dc = ((t >> 16) & 0xff) - 16;
                const int rr = pr + dr, cc = pc + dc;
                const bool ok = pv && t >= 0 && rr >= 0 && rr < H && cc >= 0 && cc < W;
                av = ok ? in[(rr * W + cc) * istride + ic0 + c] : 0.f;
            }
            const float* wrow = wl + k * NS + i16;
#pragma unroll
            for (int n = 0; n < NR; n++)
                acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av, wrow[n * 16], acc[n], 0, 0, 0);
        }
#pragma unroll
        for (int n = 0; n < NR; n++) {
            const int ch = n * 16 + i16;
            if (ch >= cout) continue;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int q = s * 16 + kq * 4 + r;
                if (q >= HW) continue;
                float v = acc[n][r] + bz[n];
                float* o = out + q * ostride + oc0 + ch;
                if (residual) v += *o;
                *o = v;
            }
        }
    }
}

template <int KS>
__device__ __forceinline__ void conv_lds_any(const float* in, int istride, int ic0, int cin, int d, int H, int W,
                                             const float* wl, int Kpad, int NS, const int* ktab, float* out,
                                             int ostride, int oc0, int cout, const float* bias, bool residual) {
    const int nr = (cout + 15) / 16;
    if (nr == 1)
        conv_lds<KS, 1>(in, istride, ic0, cin, d, H, W, wl, Kpad, NS, ktab, out, ostride, oc0, cout, bias, residual);
    else if (nr == 2)
        conv_lds<KS, 2>(in, istride, ic0, cin, d, H, W, wl, Kpad, NS, ktab, out, ostride, oc0, cout, bias, residual);
    else if (nr == 3)
        conv_lds<KS, 3>(in, istride, ic0, cin, d, H, W, wl, Kpad, NS, ktab, out, ostride, oc0, cout, bias, residual);
    else
        conv_lds<KS, 4>(in, istride, ic0, cin, d, H, W, wl, Kpad, NS, ktab, out, ostride, oc0, cout, bias, residual);
}

// k -> (dr, dc, c) table of a 3x3 dilation-d conv over cin channels, -1 beyond K
__device__ __forceinline__ void build_ktab(int* ktab, int cin, int d, int Kpad) {
    for (int k = threadIdx.x; k < Kpad; k += NT) {
        int t = -1;
        if (k < 9 * cin) {
            const int tap = k / cin, c = k - tap * cin;
            const int kh = tap / 3, kw = tap - kh * 3;
            t = (((kh - 1) * d + 16) << 24) | (((kw - 1) * d + 16) << 16) | c;
        }
        ktab[k] = t;
    }
}

}  // namespace

__device__ __forceinline__ int mask_pos_(int m, int p, int c, int wc, int W, int D) {
    const int pr = p / wc, pc = p - pr * wc;
    if (m < 2) {
        const int half = c >= D ? 1 : 0;
        const int ch = c - half * D;
        const int dr = half;
        const int dcol = (m == 0) ? half : 1 - half;
        return ((2 * pr + dr) * W + (2 * pc + dcol)) * D + ch;
    }
    const int ch = (m == 2) ? 2 * c : 2 * c + 1;
    return (pr * W + pc) * D + ch;
}

__global__ __launch_bounds__(NT) void k_net_lds(NetLdsArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int img = blockIdx.x, net = blockIdx.y;
    const int H = a.hc, W = a.wc, HW = H * W;
    const int nk = a.nk, gc = a.gc;
    const int SY = a.sy, S1 = a.s1, S2 = a.s2;   // S2 covers max(gc, nk, dc1, dc2) channels
    float* Y = reinterpret_cast<float*>(smem + a.off_y);
    float* T1 = reinterpret_cast<float*>(smem + a.off_t1);
    float* T2 = reinterpret_cast<float*>(smem + a.off_t2);
    float* WL = reinterpret_cast<float*>(smem + a.off_w);
    int* KT = reinterpret_cast<int*>(smem + a.off_k);
    double* red = reinterpret_cast<double*>(smem);
    const float* P = a.params;
    const int* off = a.offs + net * a.offs_per_net;   // see NetLdsArgs
    const bool ln = a.ln != 0;
    float mu = 0.f, rstd = 1.f;

    // gather u1c (mask compress, :720-759) straight from u into T2 (stride S2)
    {
        const float* ub = a.u + (size_t)img * a.H * a.W * a.D;
        const int n = HW * a.dc1;
        for (int e = threadIdx.x; e < n; e += NT) {
            const int p = e / a.dc1, c = e - p * a.dc1;
            T2[p * S2 + c] = ub[mask_pos_(a.mask, p, c, W, a.W, a.D)];
        }
    }
    // conv_in (3x3, dc1 -> nk)
    {
        const int K = 9 * a.dc1, Kpad = (K + 3) / 4 * 4, NS = ns_of(nk);
        stage_w(P + off[0], K, nk, Kpad, NS, WL);
        build_ktab(KT, a.dc1, 1, Kpad);
        __syncthreads();
        conv_lds_any<3>(T2, S2, 0, a.dc1, 1, H, W, WL, Kpad, NS, KT, Y, SY, 0, nk, P + off[1], false);
        __syncthreads();
    }
    const int RB0 = 2;   // offs: [conv_in_k, conv_in_b, per rb: 10 + 2*nbr, ln_out_g, ln_out_b, conv_out_k, conv_out_b]
    const int per_rb = 10 + 2 * a.nbr;
    for (int r = 0; r < a.R; r++) {
        const int* o = off + RB0 + r * per_rb;
        // LN1(LReLU(y)) -> T2 (scratch), conv_a (1x1 nk->nk) -> T1
        if (ln) ln_stats(Y, SY, HW, nk, red, mu, rstd);
        ln_apply(Y, SY, T2, S2, HW, 0, nk, nk, mu, rstd, ln ? P + o[0] : nullptr, ln ? P + o[1] : nullptr, ln);
        {
            const int Kpad = (nk + 3) / 4 * 4, NS = ns_of(nk);
            stage_w(P + o[2], nk, nk, Kpad, NS, WL);
            __syncthreads();
            conv_lds_any<1>(T2, S2, 0, nk, 1, H, W, WL, Kpad, NS, KT, T1, S1, 0, nk, P + o[3], false);
            __syncthreads();
        }
        // LN2(LReLU(t1)) in place on the channel windows the grouped branches read
        if (ln) ln_stats(T1, S1, HW, nk, red, mu, rstd);
        for (int wi = 0; wi < a.nwin; wi++)
            ln_apply(T1, S1, T1, S1, HW, a.win_off[wi], a.win_len[wi], nk, mu, rstd, ln ? P + o[4] : nullptr,
                     ln ? P + o[5] : nullptr, ln);
        __syncthreads();
        // grouped dilated branches -> T2[:, out_off : out_off + cout]
        for (int bi = 0; bi < a.nbr; bi++) {
            const int cin = a.br_cin[bi], cout = a.br_cout[bi], d = a.br_dil[bi];
            const int K = 9 * cin, Kpad = (K + 3) / 4 * 4, NS = ns_of(cout);
            stage_w(a.aux + o[10 + 2 * bi], K, cout, Kpad, NS, WL);
            build_ktab(KT, cin, d, Kpad);
            __syncthreads();
            conv_lds_any<3>(T1, S1, a.br_cin_off[bi], cin, d, H, W, WL, Kpad, NS, KT, T2, S2, a.br_out_off[bi], cout,
                            a.aux + o[11 + 2 * bi], false);
            __syncthreads();
        }
        // LN3(LReLU(t2)) in place, conv_b (1x1 gc->nk) + shortcut -> Y
        if (ln) ln_stats(T2, S2, HW, gc, red, mu, rstd);
        ln_apply(T2, S2, T2, S2, HW, 0, gc, gc, mu, rstd, ln ? P + o[6] : nullptr, ln ? P + o[7] : nullptr, ln);
        {
            const int Kpad = (gc + 3) / 4 * 4, NS = ns_of(nk);
            stage_w(P + o[8], gc, nk, Kpad, NS, WL);
            __syncthreads();
            conv_lds_any<1>(T2, S2, 0, gc, 1, H, W, WL, Kpad, NS, KT, Y, SY, 0, nk, P + o[9], true);
            __syncthreads();
        }
    }
    // LN_out(LReLU(y)) in place, conv_out (3x3 nk -> dc2) -> T2 -> global
    {
        const int* o = off + RB0 + a.R * per_rb;
        if (ln) ln_stats(Y, SY, HW, nk, red, mu, rstd);
        ln_apply(Y, SY, Y, SY, HW, 0, nk, nk, mu, rstd, ln ? P + o[0] : nullptr, ln ? P + o[1] : nullptr, ln);
        const int K = 9 * nk, Kpad = (K + 3) / 4 * 4, NS = ns_of(a.dc2);
        stage_w(P + o[2], K, a.dc2, Kpad, NS, WL);
        build_ktab(KT, nk, 1, Kpad);
        __syncthreads();
        conv_lds_any<3>(Y, SY, 0, nk, 1, H, W, WL, Kpad, NS, KT, T2, S2, 0, a.dc2, P + o[3], false);
        __syncthreads();
        float* dst = a.so[net] + (size_t)img * HW * a.dc2;
        const int n = HW * a.dc2;
        for (int e = threadIdx.x; e < n; e += NT) {
            const int p = e / a.dc2, c = e - p * a.dc2;
            dst[e] = T2[p * S2 + c];
        }
    }
}

void launch_net_lds(const NetLdsArgs& a, int B, int lds, hipStream_t st) {
    hipLaunchKernelGGL(k_net_lds, dim3(B, 2), dim3(NT), lds, st, a);
}

}  // namespace cnf
