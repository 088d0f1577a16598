// cnf_netlds.hip — one workgroup computes a whole s,t network (net A or net b of one coupling
// layer, conv_cINN_make_model.py:1076-1213 + conv_cINN_base_functions.py:330-627) for ONE image
// with every activation resident in LDS. Used for the layers whose activations fit the 160 KiB
// LDS of a CU (the compressed images of 16x16 and below at cfg2); the ~11 launches of the
// streamed path collapse into one.
//
// LDS: reduction slots | Y (residual stream, nk ch) | T1 (nk ch) | T2 (concat of the grouped
// branches, gc ch; also the normalised input of conv_a and the gathered u1c of conv_in) | W
// (packed weights of the conv being run) | K (tap / quad table). Pixel strides are == 8 (mod 16)
// floats so the channel-quad ds_read_b128 A reads are bank-conflict free.
//
// LayerNorm statistics (per image over H*W*C, conv_cINN_base_functions.py:357) are produced in
// the epilogue of the conv(s) that write the tensor: every lane accumulates shifted fp32 sums of
// LeakyReLU(out) (shift = a wave-uniform sample value), each wave reduces them once per tensor into
// its LDS slot, and after the producer's barrier every wave merges the NW slots — no extra pass.
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

#include "cnf_device.h"

namespace cnf {

#include "cnf_netlds_shapes.inc"   // shape-specialised instantiations (gen_netlds_shapes.py)

namespace {

#ifndef CNF_NETLDS_NW
#define CNF_NETLDS_NW 8
#endif
constexpr int NW = CNF_NETLDS_NW;   // waves per workgroup (one workgroup per CU: LDS-bound)
#ifndef CNF_NETLDS_NOKS
#define CNF_NETLDS_NOKS 0   // experiment knob: no K-split instantiations
#endif
#ifndef CNF_NETLDS_PAIR
#define CNF_NETLDS_PAIR 1
#endif
constexpr bool PAIR = CNF_NETLDS_PAIR != 0;   // two 16-pixel subtiles per wave and pass
constexpr int NT = NW * 64;         // threads
#ifndef CNF_CQ
#define CNF_CQ 2   // 3x3 groups per chunk (conv3q_lds)
#endif

// LeakyReLU(0.3) as max(x, 0.3x) (2 VALU ops; equal to the select form for every finite x)
__device__ __forceinline__ float lrelu_(float x) { return lrelu(x); }   // (cnf_device.h)

__device__ __forceinline__ float wsum_f(float v) { return wave_sum_f(v); }   // DPP (cnf_device.h)
__device__ __forceinline__ double wsum_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ---------------------------------------------------------------------------------------------
// LN statistics produced in conv epilogues. Every lane accumulates fp32 sums of LeakyReLU(out) - K,
// K a wave-uniform sample value of the tensor (so sum (x-K)^2 does not cancel), across every conv
// that produces the tensor (the grouped branches share one LStat); the value count is kept as a
// wave-uniform scalar. Once per tensor each wave reduces its sums (DPP) and lane 0 writes
// (K, S1, S2, n) to the wave's 16-byte LDS slot: no read-modify-write, no fp64.
// ---------------------------------------------------------------------------------------------
struct LStat {
    float K, s1, s2;
    int cnt;     // values added (wave-uniform)
    bool kset;   // K chosen (wave-uniform)
};
__device__ __forceinline__ void lst_reset(LStat& a) {
    a.K = 0.f;
    a.s1 = 0.f;
    a.s2 = 0.f;
    a.cnt = 0;
    a.kset = false;
}
// shift = LeakyReLU of lane 0's value at the wave's first output (call in wave-uniform control flow)
__device__ __forceinline__ void lst_setk(LStat& a, float v) {
    if (a.kset) return;
    a.K = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, lrelu_(v))));
    a.kset = true;
}
__device__ __forceinline__ void lst_add(LStat& a, float v) {
    const float d = lrelu_(v) - a.K;
    a.s1 += d;
    a.s2 = fmaf(d, d, a.s2);
}
// wave-reduce the lane sums and write (K, S1, S2, n) to this wave's slot (every wave, once per tensor)
__device__ __forceinline__ void lst_flush(const LStat& a, float* slots) {
#ifdef CNF_ABL_NOSTATS
    return;
#endif
    const float s1 = wsum_f(a.s1), s2 = wsum_f(a.s2);
    if ((threadIdx.x & 63) == 0)
        *reinterpret_cast<f4*>(slots + 4 * (threadIdx.x >> 6)) = f4{a.K, s1, s2, (float)a.cnt};
}
// (mean, rstd) of the tensor from the NW slots (every wave, after the producer's barrier): every
// lane reads all slots (uniform-address LDS broadcasts, one round trip) and merges them in the same
// fixed order, so every lane of every wave gets bitwise the same pair. Per wave n_w, mean_w,
// M2_w = S2 - S1^2/n; then mean = sum n_w mean_w / N, M2 = sum M2_w + n_w (mean_w - mean)^2 (fp32;
// the shifted per-wave sums keep it well conditioned).
__device__ __forceinline__ void lst_final(const float* slots, float& mu, float& rstd) {
#ifdef CNF_ABL_NOSTATS
    mu = 0.f;
    rstd = 1.f;
    return;
#endif
    f4 q[NW];
#pragma unroll
    for (int w = 0; w < NW; w++) q[w] = *reinterpret_cast<const f4*>(slots + 4 * w);
    float n[NW], m[NW], M2[NW];
    float N = 0.f, S = 0.f;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        n[w] = q[w][3];
        const float r = n[w] > 0.f ? q[w][1] * __builtin_amdgcn_rcpf(n[w]) : 0.f;
        m[w] = q[w][0] + r;
        M2[w] = fmaxf(fmaf(-q[w][1], r, q[w][2]), 0.f);
        N += n[w];
        S = fmaf(n[w], m[w], S);
    }
    const float iN = __builtin_amdgcn_rcpf(N);
    const float mean = S * iN;
    float M = 0.f;
#pragma unroll
    for (int w = 0; w < NW; w++) {
        const float d = m[w] - mean;
        M += fmaf(n[w] * d, d, M2[w]);
    }
    mu = mean;
    rstd = __builtin_amdgcn_rsqf(fmaf(M, iN, LN_EPS));
}

// dst[p][c] = LN(LeakyReLU(src[p][c])) for channels [c0, c0+nc) of a C_ln-channel LN tensor;
// gamma/beta are per (p, c) over C_ln channels (global, L2-resident). dst may alias src.
// Quad-aligned windows take a float4 path with up to 8 gamma + 8 beta float4 loads in flight.
__device__ __forceinline__ void ln_apply(const float* src, int sstride, float* dst, int dstride, int HW, int c0,
                                         int nc, int C_ln, float mu, float rstd, const float* __restrict__ g,
                                         const float* __restrict__ b, bool ln) {
    const int n = HW * nc;
    const float nmr = -mu * rstd;
    if (((sstride | dstride | nc | c0 | C_ln) & 3) == 0) {
        const int n4 = n >> 2, C4 = nc >> 2;
        const bool full = (c0 == 0 && nc == C_ln);   // gamma/beta contiguous over the whole image
        const f4* g4 = reinterpret_cast<const f4*>(g);
        const f4* b4 = reinterpret_cast<const f4*>(b);
        constexpr int UV = 8;
        for (int base = 0; base < n4; base += NT * UV) {
            f4 gv[UV], bv[UV];
            if (ln) {
#pragma unroll
                for (int u = 0; u < UV; u++) {
                    const int i = base + u * NT + (int)threadIdx.x;
                    const int p = i / C4, c = (i - p * C4) << 2;
                    const int gi = full ? i : (p * C_ln + c0 + c) >> 2;
                    gv[u] = i < n4 ? g4[gi] : f4{0.f, 0.f, 0.f, 0.f};
                    bv[u] = i < n4 ? b4[gi] : f4{0.f, 0.f, 0.f, 0.f};
                }
            }
#pragma unroll
            for (int u = 0; u < UV; u++) {
                const int i = base + u * NT + (int)threadIdx.x;
                if (i >= n4) continue;
                const int p = i / C4, c = c0 + ((i - p * C4) << 2);
                f4 x = *reinterpret_cast<const f4*>(src + p * sstride + c);
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float t = lrelu_(x[j]);
                    x[j] = ln ? fmaf(fmaf(t, rstd, nmr), gv[u][j], bv[u][j]) : t;
                }
                *reinterpret_cast<f4*>(dst + p * dstride + c) = x;
            }
        }
        return;
    }
    constexpr int US = 8;
    for (int base = 0; base < n; base += NT * US) {
        float xv[US], gv[US], bv[US];
        int pp[US], cc[US];
#pragma unroll
        for (int u = 0; u < US; u++) {
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
        for (int u = 0; u < US; u++) {
            const int e = base + u * NT + threadIdx.x;
            if (e >= n) continue;
            const float t = lrelu_(xv[u]);
            dst[pp[u] * dstride + c0 + cc[u]] = ln ? fmaf(fmaf(t, rstd, nmr), gv[u], bv[u]) : t;
        }
    }
}

// training forward: a raw LDS tensor [HW][sstride] (C channels) to its dense [HW][C] save slot
__device__ __forceinline__ void save_tensor(const float* src, int sstride, int HW, int C, float* __restrict__ dst) {
    if (((C | sstride) & 3) == 0) {
        const int C4 = C >> 2, n4 = HW * C4;
        for (int i = threadIdx.x; i < n4; i += NT) {
            const int p = i / C4, c = (i - p * C4) << 2;
            *reinterpret_cast<f4*>(dst + p * C + c) = *reinterpret_cast<const f4*>(src + p * sstride + c);
        }
        return;
    }
    const int n = HW * C;
    for (int e = threadIdx.x; e < n; e += NT) {
        const int p = e / C, c = e - p * C;
        dst[e] = src[p * sstride + c];
    }
}

// Register prefetch of the next full-width LayerNorm's gamma/beta quads i = u*NT + tid (u < GPF),
// issued before the conv that produces the tensor and consumed by ln_full after it; quads beyond
// the window are loaded on demand.
constexpr int GPF = 4;
struct LnPre {
    f4 g[GPF], b[GPF];
};
__device__ __forceinline__ void lnp_load(LnPre& L, const float* __restrict__ g, const float* __restrict__ b, int n4) {
    const f4* g4 = reinterpret_cast<const f4*>(g);
    const f4* b4 = reinterpret_cast<const f4*>(b);
#pragma unroll
    for (int u = 0; u < GPF; u++) {
        const int i = u * NT + (int)threadIdx.x;
        L.g[u] = i < n4 ? g4[i] : f4{0.f, 0.f, 0.f, 0.f};
        L.b[u] = i < n4 ? b4[i] : f4{0.f, 0.f, 0.f, 0.f};
    }
}
// dst = LN(LeakyReLU(src)) over a full-width C-channel tensor (C % 4 == 0; dst may alias src)
__device__ __forceinline__ void ln_full(const float* src, int sstride, float* dst, int dstride, int HW, int C,
                                        float mu, float rstd, const LnPre& L, const float* __restrict__ g,
                                        const float* __restrict__ b) {
    const int C4 = C >> 2, n4 = HW * C4;
    const float nmr = -mu * rstd;
#pragma unroll
    for (int u = 0; u < GPF; u++) {
        const int i = u * NT + (int)threadIdx.x;
        if (i < n4) {
            const int p = i / C4, c = (i - p * C4) << 2;
            f4 x = *reinterpret_cast<const f4*>(src + p * sstride + c);
#pragma unroll
            for (int j = 0; j < 4; j++) x[j] = fmaf(fmaf(lrelu_(x[j]), rstd, nmr), L.g[u][j], L.b[u][j]);
            *reinterpret_cast<f4*>(dst + p * dstride + c) = x;
        }
    }
    const f4* g4 = reinterpret_cast<const f4*>(g);
    const f4* b4 = reinterpret_cast<const f4*>(b);
    for (int i0 = GPF * NT; i0 < n4; i0 += NT * 8) {
        f4 gv[8], bv[8], xv[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int i = i0 + u * NT + (int)threadIdx.x;
            const int p = i / C4, c = (i - p * C4) << 2;
            gv[u] = i < n4 ? g4[i] : f4{0.f, 0.f, 0.f, 0.f};
            bv[u] = i < n4 ? b4[i] : f4{0.f, 0.f, 0.f, 0.f};
            xv[u] = i < n4 ? *reinterpret_cast<const f4*>(src + p * sstride + c) : f4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int i = i0 + u * NT + (int)threadIdx.x;
            if (i >= n4) continue;
            const int p = i / C4, c = (i - p * C4) << 2;
            f4 x = xv[u];
#pragma unroll
            for (int j = 0; j < 4; j++) x[j] = fmaf(fmaf(lrelu_(x[j]), rstd, nmr), gv[u][j], bv[u][j]);
            *reinterpret_cast<f4*>(dst + p * dstride + c) = x;
        }
    }
}

// In-place LN(LeakyReLU) over the disjoint channel windows of buf (the grouped branches' inputs)
// in ONE pass: the elements of all windows are enumerated together, so every gamma/beta load of
// a thread is in flight at once (one L2 round trip instead of one per window).
__device__ __forceinline__ void ln_windows(float* buf, int stride, int HW, int C_ln, int nwin, const int* woff,
                                           const int* wlen, float mu, float rstd, const float* __restrict__ g,
                                           const float* __restrict__ b, bool ln) {
    int total = 0;
    for (int k = 0; k < nwin; k++) total += HW * wlen[k];
    const float nmr = -mu * rstd;
    constexpr int US = 8;
    for (int base = 0; base < total; base += NT * US) {
        int pos[US], gi[US];
        float xv[US], gv[US], bv[US];
#pragma unroll
        for (int u = 0; u < US; u++) {
            int e = base + u * NT + (int)threadIdx.x;
            pos[u] = -1;
            gi[u] = 0;
            if (e < total) {
                for (int k = 0; k < nwin; k++) {
                    const int m = HW * wlen[k];
                    if (e < m) {
                        const int p = e / wlen[k], c = woff[k] + (e - p * wlen[k]);
                        pos[u] = p * stride + c;
                        gi[u] = p * C_ln + c;
                        break;
                    }
                    e -= m;
                }
            }
            xv[u] = pos[u] >= 0 ? buf[pos[u]] : 0.f;
            if (ln) {
                gv[u] = g[gi[u]];
                bv[u] = b[gi[u]];
            }
        }
#pragma unroll
        for (int u = 0; u < US; u++) {
            if (pos[u] < 0) continue;
            const float t = lrelu_(xv[u]);
            buf[pos[u]] = ln ? fmaf(fmaf(t, rstd, nmr), gv[u], bv[u]) : t;
        }
    }
}

// Register prefetch of the next conv's pre-packed weight image: loaded before the current conv's
// MFMA loop, written to LDS after the barrier that retires the current conv.
constexpr int WPF = NW >= 16 ? 2 : 4;   // float4 per thread -> up to WPF*NT*4 floats
struct WPre {
    f4 v[WPF];
    int n4;
};
__device__ __forceinline__ void wpf_load(WPre& w, const float* __restrict__ src, int n) {
    w.n4 = n >> 2;
    const f4* s4 = reinterpret_cast<const f4*>(src);
#pragma unroll
    for (int u = 0; u < WPF; u++) {
        const int i = u * NT + (int)threadIdx.x;
        w.v[u] = i < w.n4 ? s4[i] : f4{0.f, 0.f, 0.f, 0.f};
    }
}
__device__ __forceinline__ void wpf_store(const WPre& w, float* dst, const float* __restrict__ src) {
    f4* d4 = reinterpret_cast<f4*>(dst);
#pragma unroll
    for (int u = 0; u < WPF; u++) {
        const int i = u * NT + (int)threadIdx.x;
        if (i < w.n4) d4[i] = w.v[u];
    }
    // images larger than the prefetch window are finished directly
    const f4* s4 = reinterpret_cast<const f4*>(src);
    for (int i = WPF * NT + (int)threadIdx.x; i < w.n4; i += NT) d4[i] = s4[i];
}

// ---------------------------------------------------------------------------------------------
// convolutions from LDS (MFMA v_mfma_f32_16x16x4f32). Every conv takes two 16-pixel subtiles per
// wave and pass (they share the B reads); the epilogue adds bias (+ residual), stores, and
// (slots != null) accumulates the LN statistics of LeakyReLU(out).
// ---------------------------------------------------------------------------------------------
template <int NR>
struct Epi {
    float bz[NR];
    bool chv[NR];
    int cout;
    __device__ __forceinline__ void init(const float* __restrict__ bias, int cout_) {
        cout = cout_;
        const int i16 = threadIdx.x & 15;
#pragma unroll
        for (int n = 0; n < NR; n++) {
            const int ch = n * 16 + i16;
            chv[n] = ch < cout;
            const float b = bias != nullptr ? bias[chv[n] ? ch : 0] : 0.f;   // unconditional LDS read
            bz[n] = chv[n] ? b : 0.f;
        }
    }
    // write subtile sb of acc; out points at channel oc0 of pixel 0
    __device__ __forceinline__ void store(const f4 (&acc)[NR], int sb, int HW, float* out, int ostride, bool residual,
                                          bool stats, LStat& st) {
#ifdef CNF_ABL_NOEPI
        if (sb >= 0) return;
#endif
#ifdef CNF_ABL_NOSTATS
        stats = false;
#endif
        if (stats) st.cnt += min(16, HW - sb * 16) * cout;
        const int i16 = threadIdx.x & 15, kq = (threadIdx.x & 63) >> 4;
#pragma unroll
        for (int n = 0; n < NR; n++) {
            if (!chv[n]) continue;
#pragma unroll
            for (int r = 0; r < 4; r++) {
                const int q = sb * 16 + kq * 4 + r;
                if (q >= HW) continue;
                float* o = out + q * ostride + n * 16 + i16;
                float v = acc[n][r] + bz[n];
                if (residual) v += *o;
                *o = v;
                if (stats) lst_add(st, v);
            }
        }
    }
};

// K-split for images of at most NW/2 subtiles (4x4 .. 8x8 compressed images): instead of leaving
// most waves idle, wave w takes subtile w % nsub and K slice w / nsub of KS = NW / nsub; slices
// 1..KS-1 park their partial accumulators in LDS, and after one barrier slice 0 sums them in a fixed
// order (bitwise reproducible) and runs the epilogue. Two buffers alternate (par), so a conv that
// follows without a barrier of its own (the grouped branches, the tap-GEMM chunks) never overwrites
// partials still being read.
struct KSplit {
    float* buf;   // two buffers of (NW - 1) x 5 blocks x 64 lanes x 4 floats (null: no K-split)
    int par;
};
constexpr int KS_BUF = (NW - 1) * 5 * 64 * 4;   // floats per buffer
// the K-split pays when at least half the waves would idle and there are K groups to split
__device__ __forceinline__ bool ks_on(const KSplit& ks, int nsub, int G) {
    return ks.buf != nullptr && 2 * nsub <= NW && G >= 2;
}
__device__ __forceinline__ void ks_slice(int nsub, int G, int& s, int& k, int& KS, int& glo, int& ghi) {
    const int wave = threadIdx.x >> 6;
    KS = min(NW / nsub, G);
    s = wave % nsub;
    k = wave / nsub;
    glo = k < KS ? (k * G) / KS : 0;
    ghi = k < KS ? ((k + 1) * G) / KS : 0;
}
template <int NR>
__device__ __forceinline__ void ks_finish(f4 (&acc)[NR], int s, int k, int KS, int nsub, const KSplit& ks,
                                          Epi<NR>& ep, int HW, float* out, int ostride, bool residual, bool stats,
                                          LStat& st) {
    const int lane = threadIdx.x & 63;
    float* b = ks.buf + ks.par * KS_BUF;
    if (k > 0 && k < KS) {
#pragma unroll
        for (int n = 0; n < NR; n++)
            *reinterpret_cast<f4*>(b + ((((k - 1) * nsub + s) * NR + n) * 64 + lane) * 4) = acc[n];
    }
    lds_barrier();
    if (k == 0) {
        for (int kk = 1; kk < KS; kk++)
#pragma unroll
            for (int n = 0; n < NR; n++)
                acc[n] += *reinterpret_cast<const f4*>(b + ((((kk - 1) * nsub + s) * NR + n) * 64 + lane) * 4);
        if (stats) lst_setk(st, acc[0][0] + ep.bz[0]);
        ep.store(acc, s, HW, out, ostride, residual, stats, st);
    }
}

// 1x1 conv: A = in[p][0..cin) (pixel stride == 8 mod 16), PK_1X1 image wl ([g][q][j][s], lane
// (i, q) holds channels 16g + 4q + s at k-step s); out[p][n] (+)= bias + A.B. nsj / nb0: column
// count of the packed image and first 16-column block this call computes (column-chunked calls).
template <int NR>
__device__ __forceinline__ void conv1_lds(const float* in, int istride, int cin, int HW, const float* wl, float* out,
                                          int ostride, int cout, const float* __restrict__ bias, bool residual,
                                          LStat& st, bool stats, int nsj, int nb0, const KSplit& ks) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, kq = lane >> 4;
    const int nsub = (HW + 15) >> 4;
    const int G = (cin + 15) >> 4;
    Epi<NR> ep;
    ep.init(bias, cout);
    if (ks_on(ks, nsub, G)) {
        int s, k, KS, glo, ghi;
        ks_slice(nsub, G, s, k, KS, glo, ghi);
        f4 acc[NR];
#pragma unroll
        for (int n = 0; n < NR; n++) acc[n] = f4{0.f, 0.f, 0.f, 0.f};
        const int pa = s * 16 + i16;
        const bool pva = pa < HW;
        for (int g = glo; g < ghi; g++) {
            const int c0 = 16 * g + 4 * kq;
            f4 a0 = (pva && c0 < cin) ? *reinterpret_cast<const f4*>(in + pa * istride + c0) : f4{0.f, 0.f, 0.f, 0.f};
            if (c0 + 4 > cin) {
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (c0 + j >= cin) a0[j] = 0.f;
            }
            const float* brow = wl + ((g * 4 + kq) * nsj + i16) * 4 + nb0 * 64;
            f4 bq[NR];
#pragma unroll
            for (int n = 0; n < NR; n++) bq[n] = *reinterpret_cast<const f4*>(brow + n * 64);
#pragma unroll
            for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
                for (int n = 0; n < NR; n++) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s4], bq[n][s4], acc[n], 0, 0, 0);
        }
        ks_finish<NR>(acc, s, k, KS, nsub, ks, ep, HW, out, ostride, residual, stats, st);
        return;
    }
    for (int s0 = wave; s0 < nsub; s0 += (PAIR ? 2 : 1) * NW) {
        const int s1 = s0 + NW;
        const bool v1 = PAIR && s1 < nsub;
        const int pa = s0 * 16 + i16, pb = s1 * 16 + i16;
        const bool pva = pa < HW, pvb = v1 && pb < HW;
        f4 acc0[NR], acc1[NR];
#pragma unroll
        for (int n = 0; n < NR; n++) {
            acc0[n] = f4{0.f, 0.f, 0.f, 0.f};
            acc1[n] = f4{0.f, 0.f, 0.f, 0.f};
        }
        for (int g = 0; g < G; g++) {
            const int c0 = 16 * g + 4 * kq;
            const bool cv = c0 < cin;
            f4 a0 = (pva && cv) ? *reinterpret_cast<const f4*>(in + pa * istride + c0) : f4{0.f, 0.f, 0.f, 0.f};
            f4 a1 = (pvb && cv) ? *reinterpret_cast<const f4*>(in + pb * istride + c0) : f4{0.f, 0.f, 0.f, 0.f};
            if (c0 + 4 > cin) {   // ragged channel tail (cin % 4 != 0)
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (c0 + j >= cin) {
                        a0[j] = 0.f;
                        a1[j] = 0.f;
                    }
            }
            const float* brow = wl + ((g * 4 + kq) * nsj + i16) * 4 + nb0 * 64;
            f4 bq[NR];
#pragma unroll
            for (int n = 0; n < NR; n++) bq[n] = *reinterpret_cast<const f4*>(brow + n * 64);
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int n = 0; n < NR; n++) {
                    acc0[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s], bq[n][s], acc0[n], 0, 0, 0);
                    acc1[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[s], bq[n][s], acc1[n], 0, 0, 0);
                }
        }
        if (stats) lst_setk(st, acc0[0][0] + ep.bz[0]);
        ep.store(acc0, s0, HW, out, ostride, residual, stats, st);
        if (v1) ep.store(acc1, s1, HW, out, ostride, residual, stats, st);
    }
}

// MAXNR: the widest output block count the instantiation supports (wider is compiled out, which
// keeps the narrow instantiation's register allocation small; the host picks MAXNR per layer)
template <int MAXNR>
__device__ __forceinline__ void conv1_any(const float* in, int istride, int cin, int HW, const float* wl, float* out,
                                          int ostride, int cout, const float* bias, bool residual, LStat& st, bool stats,
                                          const KSplit& ks, int nsj = 0, int nb0 = 0) {
    const int nr = (cout + 15) / 16;
    if (nsj == 0) nsj = 16 * nr;
    if (MAXNR <= 2 || nr <= 2) {
        if (nr == 1)
            conv1_lds<1>(in, istride, cin, HW, wl, out, ostride, cout, bias, residual, st, stats, nsj, nb0, ks);
        else
            conv1_lds<2>(in, istride, cin, HW, wl, out, ostride, cout, bias, residual, st, stats, nsj, nb0, ks);
        return;
    }
    switch (nr) {
        case 3: conv1_lds<MAXNR >= 3 ? 3 : 2>(in, istride, cin, HW, wl, out, ostride, cout, bias, residual, st, stats, nsj, nb0, ks); break;
        case 4: conv1_lds<MAXNR >= 4 ? 4 : 2>(in, istride, cin, HW, wl, out, ostride, cout, bias, residual, st, stats, nsj, nb0, ks); break;
        default: conv1_lds<MAXNR >= 5 ? 5 : 2>(in, istride, cin, HW, wl, out, ostride, cout, bias, residual, st, stats, nsj, nb0, ks); break;
    }
}

// quad table of a PK_Q4 conv: entry qd = tap*(cin/4) + cq -> packed (dr+32 | dc+32 << 6 | c << 12),
// c = ic0 + 4cq; -1 for the padding quads of the last group
__device__ __forceinline__ void build_qtab(int* qt, int cin, int ic0, int d) {
    const int cpq = cin >> 2, nq = 9 * cpq, nq4 = (nq + 3) & ~3;
    for (int qd = threadIdx.x; qd < nq4; qd += NT) {
        int t = -1;
        if (qd < nq) {
            const int tap = qd / cpq, cq = qd - tap * cpq;
            const int dr = (tap / 3 - 1) * d, dc = (tap % 3 - 1) * d;
            t = (dr + 32) | ((dc + 32) << 6) | ((ic0 + 4 * cq) << 12);
        }
        qt[qd] = t;
    }
}

// 3x3 dilated conv, PK_Q4: per group g each lane reads one channel quad (tap, cq) of its shifted
// pixel with a ds_read_b128 -> 4*NR MFMAs per subtile. Groups are taken in chunks of CQ: the chunk's
// quad-table entries, then every A quad of both subtiles, are issued before its MFMAs, so the two
// dependent LDS round trips are paid once per chunk instead of once per group. Quads outside the
// image read the 16-byte zero slot zq (branch-free).
template <int NR>
__device__ __forceinline__ void conv3q_lds(const float* in, int istride, int G, int H, int W, const float* wl,
                                           const int* qt, float* out, int ostride, int cout,
                                           const float* __restrict__ bias, LStat& st, bool stats, const float* zq,
                                           const KSplit& ks) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, kq = lane >> 4;
    const int HW = H * W;
    const int nsub = (HW + 15) >> 4;
    constexpr int NSJ = 16 * NR;
    constexpr int CQ = CNF_CQ;
    Epi<NR> ep;
    ep.init(bias, cout);
    if (ks_on(ks, nsub, G)) {
        int s, k, KS, glo, ghi;
        ks_slice(nsub, G, s, k, KS, glo, ghi);
        f4 acc[NR];
#pragma unroll
        for (int n = 0; n < NR; n++) acc[n] = f4{0.f, 0.f, 0.f, 0.f};
        const int pa = s * 16 + i16;
        const bool pva = pa < HW;
        const int ra = pva ? pa / W : -4096, ca = pva ? pa - (pa / W) * W : -4096;
        for (int g = glo; g < ghi; g++) {
            const int t = qt[4 * g + kq];
            const int dr = (t & 63) - 32, dc = ((t >> 6) & 63) - 32, c = t >> 12;
            const int ya = ra + dr, xa = ca + dc;
            const bool oka = t >= 0 && (unsigned)ya < (unsigned)H && (unsigned)xa < (unsigned)W;
            const f4 a0 = *reinterpret_cast<const f4*>(oka ? in + (ya * W + xa) * istride + c : zq);
            const float* brow = wl + ((g * 4 + kq) * NSJ + i16) * 4;
            f4 bq[NR];
#pragma unroll
            for (int n = 0; n < NR; n++) bq[n] = *reinterpret_cast<const f4*>(brow + n * 64);
#pragma unroll
            for (int s4 = 0; s4 < 4; s4++)
#pragma unroll
                for (int n = 0; n < NR; n++) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[s4], bq[n][s4], acc[n], 0, 0, 0);
        }
        ks_finish<NR>(acc, s, k, KS, nsub, ks, ep, HW, out, ostride, false, stats, st);
        return;
    }
    for (int s0 = wave; s0 < nsub; s0 += (PAIR ? 2 : 1) * NW) {
        const int s1 = s0 + NW;
        const bool v1 = PAIR && s1 < nsub;
        const int pa = s0 * 16 + i16, pb = s1 * 16 + i16;
        const bool pva = pa < HW, pvb = v1 && pb < HW;
        const int ra = pva ? pa / W : -4096, ca = pva ? pa - (pa / W) * W : -4096;
        const int rb = pvb ? pb / W : -4096, cb = pvb ? pb - (pb / W) * W : -4096;
        f4 acc0[NR], acc1[NR];
#pragma unroll
        for (int n = 0; n < NR; n++) {
            acc0[n] = f4{0.f, 0.f, 0.f, 0.f};
            acc1[n] = f4{0.f, 0.f, 0.f, 0.f};
        }
        for (int g0 = 0; g0 < G; g0 += CQ) {
            int tq[CQ];
#pragma unroll
            for (int j = 0; j < CQ; j++) tq[j] = qt[4 * min(g0 + j, G - 1) + kq];
            f4 a0[CQ], a1[CQ];
#pragma unroll
            for (int j = 0; j < CQ; j++) {
                const int t = tq[j];
                const int dr = (t & 63) - 32, dc = ((t >> 6) & 63) - 32, c = t >> 12;
                const int ya = ra + dr, xa = ca + dc, yb = rb + dr, xb = cb + dc;
                const bool oka = t >= 0 && (unsigned)ya < (unsigned)H && (unsigned)xa < (unsigned)W;
                const bool okb = t >= 0 && (unsigned)yb < (unsigned)H && (unsigned)xb < (unsigned)W;
                a0[j] = *reinterpret_cast<const f4*>(oka ? in + (ya * W + xa) * istride + c : zq);
                a1[j] = *reinterpret_cast<const f4*>(okb ? in + (yb * W + xb) * istride + c : zq);
            }
#pragma unroll
            for (int j = 0; j < CQ; j++) {
                if (g0 + j < G) {
                    const float* brow = wl + (((g0 + j) * 4 + kq) * NSJ + i16) * 4;
                    f4 bq[NR];
#pragma unroll
                    for (int n = 0; n < NR; n++) bq[n] = *reinterpret_cast<const f4*>(brow + n * 64);
#pragma unroll
                    for (int s = 0; s < 4; s++)
#pragma unroll
                        for (int n = 0; n < NR; n++) {
                            acc0[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0[j][s], bq[n][s], acc0[n], 0, 0, 0);
                            acc1[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1[j][s], bq[n][s], acc1[n], 0, 0, 0);
                        }
                }
            }
        }
        if (stats) lst_setk(st, acc0[0][0] + ep.bz[0]);
        ep.store(acc0, s0, HW, out, ostride, false, stats, st);
        if (v1) ep.store(acc1, s1, HW, out, ostride, false, stats, st);
    }
}

template <int MAXNR>
__device__ __forceinline__ void conv3q_any(const float* in, int istride, int G, int H, int W, const float* wl,
                                           const int* qt, float* out, int ostride, int cout, const float* bias,
                                           LStat& st, bool stats, const float* zq, const KSplit& ks) {
    const int nr = (cout + 15) / 16;
    if (MAXNR <= 2 || nr <= 2) {
        if (nr == 1)
            conv3q_lds<1>(in, istride, G, H, W, wl, qt, out, ostride, cout, bias, st, stats, zq, ks);
        else
            conv3q_lds<2>(in, istride, G, H, W, wl, qt, out, ostride, cout, bias, st, stats, zq, ks);
        return;
    }
    if (nr == 3)
        conv3q_lds<MAXNR >= 3 ? 3 : 2>(in, istride, G, H, W, wl, qt, out, ostride, cout, bias, st, stats, zq, ks);
    else
        conv3q_lds<MAXNR >= 4 ? 4 : 2>(in, istride, G, H, W, wl, qt, out, ostride, cout, bias, st, stats, zq, ks);
}

// k -> (dr, dc, c) table of a PK_KN conv over cin channels from channel ic0; -1 beyond K
__device__ __forceinline__ void build_ktab(int* ktab, int cin, int ic0, int d, int Kpad) {
    for (int k = threadIdx.x; k < Kpad; k += NT) {
        int t = -1;
        if (k < 9 * cin) {
            const int tap = k / cin, c = k - tap * cin;
            t = (((tap / 3 - 1) * d + 32) << 24) | (((tap % 3 - 1) * d + 32) << 16) | (ic0 + c);
        }
        ktab[k] = t;
    }
}

// the tap geometry of a PK_KN conv, for decoding its tap table in registers (cin == 0: read the
// LDS table; the shape-specialised instantiations pass constants)
struct KTap {
    int cin, ic0, d;
};

// 3x3 dilated conv, PK_KN (any cin): scalar A reads through the tap table, K = 9*cin padded to 4.
// SPEC: k loop fully unrolled (constant Kpad) and entries decoded from kt instead of the table
template <int NR, bool SPEC>
__device__ __forceinline__ void conv3k_lds(const float* in, int istride, int H, int W, const float* wl, int Kpad,
                                           int NS, const int* ktab, float* out, int ostride, int cout,
                                           const float* __restrict__ bias, LStat& st, bool stats, const KSplit& ks,
                                           KTap kt) {
    // table entry k: (dr + 32) << 24 | (dc + 32) << 16 | channel, or -1 beyond K
    auto tap_of = [&](int k) -> int {
        if (!SPEC) return ktab[k];
        if (k >= 9 * kt.cin) return -1;
        const int tap = k / kt.cin, c = k - tap * kt.cin;
        return (((tap / 3 - 1) * kt.d + 32) << 24) | (((tap % 3 - 1) * kt.d + 32) << 16) | (kt.ic0 + c);
    };
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, kq = lane >> 4;
    const int HW = H * W;
    const int nsub = (HW + 15) >> 4;
    Epi<NR> ep;
    ep.init(bias, cout);
    if (ks_on(ks, nsub, Kpad >> 2)) {
        int s, k, KS, glo, ghi;
        ks_slice(nsub, Kpad >> 2, s, k, KS, glo, ghi);
        f4 acc[NR];
#pragma unroll
        for (int n = 0; n < NR; n++) acc[n] = f4{0.f, 0.f, 0.f, 0.f};
        const int pa = s * 16 + i16;
        const bool pva = pa < HW;
        const int ra = pva ? pa / W : -4096, ca = pva ? pa - (pa / W) * W : -4096;
        for (int k0 = 4 * glo; k0 < 4 * ghi; k0 += 4) {
            const int t = ktab[k0 + kq];   // runtime slice bounds: the table read beats a decode
            const int c = t & 0xffff;
            const int dr = ((t >> 24) & 0xff) - 32, dc = ((t >> 16) & 0xff) - 32;
            const int ya = ra + dr, xa = ca + dc;
            const bool oka = t >= 0 && (unsigned)ya < (unsigned)H && (unsigned)xa < (unsigned)W;
            const float a0 = oka ? in[(ya * W + xa) * istride + c] : 0.f;
            const float* wrow = wl + (k0 + kq) * NS + i16;
#pragma unroll
            for (int n = 0; n < NR; n++) acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, wrow[n * 16], acc[n], 0, 0, 0);
        }
        ks_finish<NR>(acc, s, k, KS, nsub, ks, ep, HW, out, ostride, false, stats, st);
        return;
    }
    for (int s0 = wave; s0 < nsub; s0 += (PAIR ? 2 : 1) * NW) {
        const int s1 = s0 + NW;
        const bool v1 = PAIR && s1 < nsub;
        const int pa = s0 * 16 + i16, pb = s1 * 16 + i16;
        const bool pva = pa < HW, pvb = v1 && pb < HW;
        const int ra = pva ? pa / W : -4096, ca = pva ? pa - (pa / W) * W : -4096;
        const int rb = pvb ? pb / W : -4096, cb = pvb ? pb - (pb / W) * W : -4096;
        f4 acc0[NR], acc1[NR];
#pragma unroll
        for (int n = 0; n < NR; n++) {
            acc0[n] = f4{0.f, 0.f, 0.f, 0.f};
            acc1[n] = f4{0.f, 0.f, 0.f, 0.f};
        }
        auto kstep = [&](int k0) {
            const int t = tap_of(k0 + kq);
            const int c = t & 0xffff;
            const int dr = ((t >> 24) & 0xff) - 32, dc = ((t >> 16) & 0xff) - 32;
            const int ya = ra + dr, xa = ca + dc, yb = rb + dr, xb = cb + dc;
            const bool oka = t >= 0 && (unsigned)ya < (unsigned)H && (unsigned)xa < (unsigned)W;
            const bool okb = t >= 0 && (unsigned)yb < (unsigned)H && (unsigned)xb < (unsigned)W;
            const float a0 = oka ? in[(ya * W + xa) * istride + c] : 0.f;
            const float a1 = okb ? in[(yb * W + xb) * istride + c] : 0.f;
            const float* wrow = wl + (k0 + kq) * NS + i16;
#pragma unroll
            for (int n = 0; n < NR; n++) {
                const float b = wrow[n * 16];
                acc0[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a0, b, acc0[n], 0, 0, 0);
                acc1[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(a1, b, acc1[n], 0, 0, 0);
            }
        };
        if constexpr (SPEC) {
#pragma unroll
            for (int k0 = 0; k0 < Kpad; k0 += 4) kstep(k0);
        } else {
#pragma unroll 2
            for (int k0 = 0; k0 < Kpad; k0 += 4) kstep(k0);
        }
        if (stats) lst_setk(st, acc0[0][0] + ep.bz[0]);
        ep.store(acc0, s0, HW, out, ostride, false, stats, st);
        if (v1) ep.store(acc1, s1, HW, out, ostride, false, stats, st);
    }
}

template <int MAXNR, bool SPEC>
__device__ __forceinline__ void conv3k_any(const float* in, int istride, int H, int W, const float* wl, int Kpad,
                                           int NS, const int* ktab, float* out, int ostride, int cout,
                                           const float* bias, LStat& st, bool stats, const KSplit& ks, KTap kt) {
    const int nr = (cout + 15) / 16;
    if (MAXNR <= 2 || nr <= 2) {
        if (nr == 1)
            conv3k_lds<1, SPEC>(in, istride, H, W, wl, Kpad, NS, ktab, out, ostride, cout, bias, st, stats, ks, kt);
        else
            conv3k_lds<2, SPEC>(in, istride, H, W, wl, Kpad, NS, ktab, out, ostride, cout, bias, st, stats, ks, kt);
        return;
    }
    if (nr == 3)
        conv3k_lds<MAXNR >= 3 ? 3 : 2, SPEC>(in, istride, H, W, wl, Kpad, NS, ktab, out, ostride, cout, bias, st, stats,
                                              ks, kt);
    else
        conv3k_lds<MAXNR >= 4 ? 4 : 2, SPEC>(in, istride, H, W, wl, Kpad, NS, ktab, out, ostride, cout, bias, st, stats,
                                              ks, kt);
}

// entries of the tap (PK_KN) / quad (PK_Q4) table of a 3x3 conv, rounded to 4
__device__ __forceinline__ int ktab_len(const LdsConv& cv) { return cv.fmt == PK_Q4 ? cv.kpad / 4 : cv.kpad; }

// build the table a 3x3 conv of format fmt needs (caller barriers before the conv)
__device__ __forceinline__ void conv3_table(const LdsConv& cv, int* tab, int cin, int ic0, int d) {
    if (cv.fmt == PK_Q4)
        build_qtab(tab, cin, ic0, d);
    else
        build_ktab(tab, cin, ic0, d, cv.kpad);
}
template <int MAXNR, bool SPEC = false>
__device__ __forceinline__ void conv3_run(const LdsConv& cv, const float* in, int istride, int H, int W,
                                          const float* wl, const int* tab, float* out, int ostride, int cout,
                                          const float* bias, LStat& st, bool stats, const float* zq, const KSplit& ks,
                                          KTap kt = KTap{0, 0, 0}) {
    if (cv.fmt == PK_Q4)
        conv3q_any<MAXNR>(in, istride, cv.kpad >> 4, H, W, wl, tab, out, ostride, cout, bias, st, stats, zq, ks);
    else
        conv3k_any<MAXNR, SPEC>(in, istride, H, W, wl, cv.kpad, cv.ns, tab, out, ostride, cout, bias, st, stats, ks, kt);
}

// position in u of element (pixel p, channel c) of the compressed u1c (mask compress, :720-759)
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

}  // namespace

// Diagnostic phase stamps (CNF_STAMPS=1 selects the stamping instantiation; never in timed runs):
// thread 0 of every workgroup records the shader clock (s_memtime) into an LDS array at each
// stamp point, with no barrier or memory wait of its own, so the stamps see wave 0's own timeline
// as the timed kernel runs it; workgroup (0, 0) copies its array to g_cycles at the end (with the
// realtime clock at both ends in g_stamps[0..1] for the cycle -> time scale).
__device__ long long g_stamps[256];
__device__ long long g_cycles[256];
#define STAMP(i)                                                                             \
    do {                                                                                      \
        if (STAMPS && threadIdx.x == 0) {                                                     \
            const int si_ = (i);                                                              \
            if (si_ < 128) stamp_lds[si_] = (long long)__builtin_amdgcn_s_memtime();          \
        }                                                                                     \
    } while (0)

// Shape-specialised instantiations (SID >= 0) read every shape field from the constexpr table entry
// SID (the host picks SID only when the launch's shape words match it), so strides, trip counts,
// formats and offsets are compile-time constants; SID < 0 reads them from the kernel arguments.
#define SA(f) (SID >= 0 ? kNetShapes[SID >= 0 ? SID : 0].f : a.f)

template <bool STAMPS, int MAXNR, bool KSP, int SID>
__global__ __launch_bounds__(NT) void k_net_lds(NetLdsArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int img = blockIdx.x, net = blockIdx.y;
    const int H = SA(hc), W = SA(wc), HW = H * W;
    const int nk = SA(nk), gc = SA(gc);
    const int SY = SA(sy), S1 = SA(s1), S2 = SA(s2), SU = SA(su);   // S2 covers max(gc, nk, dc2) channels
    float* slots = reinterpret_cast<float*>(smem);           // NW x (K, S1, S2, n)
    float* Y = reinterpret_cast<float*>(smem + SA(off_y));
    float* T1 = reinterpret_cast<float*>(smem + SA(off_t1));
    float* T2 = reinterpret_cast<float*>(smem + SA(off_t2));
    float* WL = reinterpret_cast<float*>(smem + SA(off_w));
    int* KT = reinterpret_cast<int*>(smem + SA(off_k));
    const float* P = a.params;
    const float* X = a.aux;
    // this net's parameter-offset table (see NetLdsArgs) copied to LDS [192, ...): every later read
    // is an LDS broadcast, so no phase drains the in-flight prefetches (vmcnt) to read an offset
    static_assert(NW * 4 * 4 + NW * 8 <= NETLDS_OTAB, "LN slots + log-det scratch overlap the offset table");
    int* otab = reinterpret_cast<int*>(smem + NETLDS_OTAB);
    // conv_in's packed image (weights + bias) prefetched first, from the offset passed as an argument:
    // its loads overlap the offset table's and the u1c gather's
    WPre pf;
    const float* ci_src = a.aux + a.ci_off[net];
    wpf_load(pf, ci_src, SA(ci).size + ((nk + 3) & ~3));
    for (int i = threadIdx.x; i < SA(offs_per_net); i += NT) otab[i] = a.offs[net * SA(offs_per_net) + i];
    // 16 zero bytes right below Y: the source of every 3x3 tap quad outside the image
    float* ZQ = reinterpret_cast<float*>(smem + SA(off_y) - 16);
    if (threadIdx.x < 4) ZQ[threadIdx.x] = 0.f;
    lds_barrier();
    const int* off = otab;
    const bool ln = SA(ln) != 0;
    LStat st;   // LN statistics of the tensor being produced
    // K-split only in the instantiation for images of at most 4 subtiles (its extra registers stay
    // out of the larger layers' kernel)
    float* ksb = KSP ? reinterpret_cast<float*>(smem + SA(off_ks)) : nullptr;
    const KSplit ks0{ksb, 0};
    float mu = 0.f, rstd = 1.f;
    // training forward: this (net, image)'s save block (LdsSave), null in inference
    float* const sv = a.save != nullptr ? a.save + ((size_t)net * gridDim.x + img) * a.save_img : nullptr;
    const int RB0 = 2;   // offs: [ci_w, ci_b, per rb: 10 + 2*nbr, ln_out_g, ln_out_b, co_w, co_b]
    const int per_rb = 10 + 2 * SA(nbr);
    auto rbo = [&](int r) { return off + RB0 + r * per_rb; };
    const int* oend = off + RB0 + SA(R) * per_rb;
    LnPre lp;
    // full-width LNs (Y: nk channels, T2: gc channels) take the prefetched path when quad-shaped
    const bool yq = ln && (nk & 3) == 0, tq = ln && (gc & 3) == 0;

    int sti = 0;
    long long* stamp_lds = reinterpret_cast<long long*>(smem + a.stamp_off);
    long long rt0 = 0;
    if (STAMPS && threadIdx.x == 0) rt0 = (long long)__builtin_amdgcn_s_memrealtime();
    STAMP(sti++);
    // packed conv images carry their bias right behind the weights (cnf_plan.cpp pack()): one
    // copy stages both, and every conv reads its bias from LDS
    auto wb = [](const LdsConv& cv, int cout) { return cv.size + ((cout + 3) & ~3); };
    // floats of all branch images of a residual block (contiguous from offs[10])
    auto brw = [&](const int* o) {
        const int l = SA(nbr) - 1;
        return o[11 + 2 * l] + ((SA(br_cout)[l] + 3) & ~3) - o[10];
    };
    // gather u1c (mask compress) into T2 (stride SU)
    if (a.pend.on == 0 && a.nz.src != nullptr) {
        // fused input preparation of the layer input (the first coupling of cnf_flow_forward_noise:
        // logit on the x channels, instance noise): the gathered half prepared, and the prepared input
        // written out (net b: the transformed half too)
        const size_t n_img = (size_t)SA(H) * SA(W) * SA(D), ib = (size_t)img * n_img;
        const float* xb = a.nz.src + ib;
        float* ub = const_cast<float*>(a.u) + ib;
        const int n = HW * SA(dc1);
        for (int e = threadIdx.x; e < n; e += NT) {
            const int p = e / SA(dc1), c = e - p * SA(dc1);
            const int pos = mask_pos_(a.mask, p, c, W, SA(W), SA(D));
            const float val = input_prep_value(xb[pos], pos % SA(D), a.nz, a.nz.off + ib + pos);
            T2[p * SU + c] = val;
            if (net == 0) ub[pos] = val;
        }
        if (net == 1) {
            const int n2 = HW * SA(dc2);
            for (int e = threadIdx.x; e < n2; e += NT) {
                const int p = e / SA(dc2), c = e - p * SA(dc2);
                const int pos = mask_pos_(a.mask ^ 1, p, c, W, SA(W), SA(D));   // the complement mask
                ub[pos] = input_prep_value(xb[pos], pos % SA(D), a.nz, a.nz.off + ib + pos);
            }
        }
    } else if (a.pend.on == 0) {
        const float* ub = a.u + (size_t)img * SA(H) * SA(W) * SA(D);
        const int n = HW * SA(dc1);
        for (int e = threadIdx.x; e < n; e += NT) {
            const int p = e / SA(dc1), c = e - p * SA(dc1);
            T2[p * SU + c] = ub[mask_pos_(a.mask, p, c, W, SA(W), SA(D))];
        }
    } else if (a.pend.comp != 0) {
        // the previous layer's coupling law is still pending and this layer conditions on exactly
        // its transformed half: the gather computes v2c_k itself; net A's workgroup stores it into
        // v_k and sums its s (layer k's log-det), net b's copies v_k's other half from u_k
        const CoupPend& q = a.pend;
        const int n_img = SA(H) * SA(W) * SA(D);
        const float* ub = q.u + (size_t)img * n_img;
        float* vb = q.v + (size_t)img * n_img;
        const size_t sb = (size_t)img * HW * SA(dc1);
        const float w = *q.tanh_w;
        const int n = HW * SA(dc1);
        // net b: the first CPF copy elements per thread loaded before the gather (one memory round
        // trip for both), stored after it
        constexpr int CPF = 4;
        const int n1 = HW * q.dc1;
        float cv[CPF];
        int cp[CPF];
        if (net == 1) {
#pragma unroll
            for (int j = 0; j < CPF; j++) {
                const int e = (int)threadIdx.x + j * NT;
                const int p = e / q.dc1, c = e - p * q.dc1;
                cp[j] = e < n1 ? mask_pos_(q.mask, p, c, W, SA(W), SA(D)) : -1;
                cv[j] = cp[j] >= 0 ? ub[cp[j]] : 0.f;
            }
        }
        float lsum = 0.f;
        for (int e = threadIdx.x; e < n; e += NT) {
            const int p = e / SA(dc1), c = e - p * SA(dc1);
            const int pos = mask_pos_(a.mask, p, c, W, SA(W), SA(D));
            const float s = w * cpl_tanh(q.s_pre[sb + e]);
            const float val = cpl_law(s, ub[pos], q.t[sb + e], q.dir);   // k_coupling's expression, bit for bit
            T2[p * SU + c] = val;
            if (net == 0) {
                vb[pos] = val;
                lsum += s;
            }
        }
        if (net == 1) {
#pragma unroll
            for (int j = 0; j < CPF; j++)
                if (cp[j] >= 0) vb[cp[j]] = cv[j];
            for (int e = (int)threadIdx.x + CPF * NT; e < n1; e += NT) {
                const int p = e / q.dc1, c = e - p * q.dc1;
                const int pos = mask_pos_(q.mask, p, c, W, SA(W), SA(D));
                vb[pos] = ub[pos];
            }
        } else {
            // wave sums -> LDS scratch [NW * 16, NW * 24); thread 0 folds them after conv_in's barrier
            const double ws = wave_sum((double)lsum);
            if ((threadIdx.x & 63) == 0) reinterpret_cast<double*>(smem + NW * 16)[threadIdx.x >> 6] = ws;
        }
    } else {
        // the previous layer's coupling law is still pending: u = v_k is computed here from u_k and
        // layer k's s, t — on the fly for the gathered half; the whole v_k (elements split between
        // the two workgroups) and layer k's log-det partial slots at the end of the kernel
        const CoupPend& q = a.pend;
        const int n_img = SA(H) * SA(W) * SA(D);
        const float* ub = q.u + (size_t)img * n_img;
        const size_t sb = (size_t)img * q.hc * q.wc * q.dc2;
        const float w = *q.tanh_w;
        auto coupled = [&](int pos, float& s) {
            const int ci = pend_index(q, pos, SA(W), SA(D));
            const float x = ub[pos];
            if (ci < 0) return x;
            s = w * cpl_tanh(q.s_pre[sb + ci]);
            return cpl_law(s, x, q.t[sb + ci], q.dir);   // k_coupling's expression, bit for bit
        };
        const int n = HW * SA(dc1);
        for (int e = threadIdx.x; e < n; e += NT) {
            const int p = e / SA(dc1), c = e - p * SA(dc1);
            float s = 0.f;
            T2[p * SU + c] = coupled(mask_pos_(a.mask, p, c, W, SA(W), SA(D)), s);
        }
    }
    // conv_in (3x3, dc1 -> nk) -> Y, LN stats of Y
    {
        conv3_table(SA(ci), KT, SA(dc1), 0, 1);
        wpf_store(pf, WL, ci_src);
        lst_reset(st);
        lds_barrier();
        if (a.pend.comp != 0 && net == 0 && threadIdx.x == 0 && a.pend.ld_part != nullptr) {   // layer k's log-det partial slots
            const double* ws = reinterpret_cast<const double*>(smem + NW * 16);
            double t = 0.0;
            for (int i = 0; i < NW; i++) t += ws[i];
            double* dst = a.pend.ld_part + (size_t)img * a.pend.np;
            dst[0] = t;
            for (int j = 1; j < a.pend.np; j++) dst[j] = 0.0;
        }
        if (SA(R) > 0)
            wpf_load(pf, X + rbo(0)[2], wb(SA(ca), nk));
        else
            wpf_load(pf, X + oend[2], wb(SA(co), SA(dc2)));
        if (yq) lnp_load(lp, P + (SA(R) > 0 ? rbo(0)[0] : oend[0]), P + (SA(R) > 0 ? rbo(0)[1] : oend[1]), HW * nk / 4);
        STAMP(sti++);
        conv3_run<MAXNR>(SA(ci), T2, SU, H, W, WL, KT, Y, SY, nk, WL + SA(ci).size, st, ln, ZQ, ks0);
        if (ln) lst_flush(st, slots);
        lds_barrier();
        STAMP(sti++);
    }
    for (int r = 0; r < SA(R); r++) {
        const int* o = rbo(r);
        // LN1(LReLU(y)) -> T2, conv_a (1x1 nk->nk) -> T1 (+ LN2 stats)
        if (ln) lst_final(slots, mu, rstd);
        if (sv != nullptr) {   // y_r and LN1_r (Y is not written again before conv_b's barriers)
            save_tensor(Y, SY, HW, nk, sv + (size_t)r * HW * nk);
            if (threadIdx.x == 0) {
                sv[a.save_st + 2 * r] = mu;
                sv[a.save_st + 2 * r + 1] = rstd;
            }
        }
        STAMP(sti++);
        if (yq)
            ln_full(Y, SY, T2, S2, HW, nk, mu, rstd, lp, P + o[0], P + o[1]);
        else
            ln_apply(Y, SY, T2, S2, HW, 0, nk, nk, mu, rstd, ln ? P + o[0] : nullptr, ln ? P + o[1] : nullptr, ln);
        STAMP(sti++);
        wpf_store(pf, WL, X + o[2]);
        STAMP(sti++);
        lds_barrier();   // every wave has read the Y slots; T2 and W are complete
        lst_reset(st);
        wpf_load(pf, X + o[10], brw(o));
        // LN2 over the whole of T1 when quad-shaped (vectorised, gamma/beta prefetched behind conv_a);
        // the branches read only their windows of it
        if (yq) lnp_load(lp, P + o[4], P + o[5], HW * nk / 4);
        STAMP(sti++);
        conv1_any<MAXNR>(T2, S2, nk, HW, WL, T1, S1, nk, WL + SA(ca).size, false, st, ln, ks0);
        if (ln) lst_flush(st, slots);
        STAMP(sti++);
        lds_barrier();
        STAMP(sti++);
        // LN2(LReLU(t1)) in place on the channel windows the grouped branches read
        if (ln) lst_final(slots, mu, rstd);
        if (sv != nullptr) {   // raw t1_r and LN2_r, before LN2 is applied in place
            save_tensor(T1, S1, HW, nk, sv + a.save_t1 + (size_t)r * HW * nk);
            if (threadIdx.x == 0) {
                sv[a.save_st + 2 * (SA(R) + r)] = mu;
                sv[a.save_st + 2 * (SA(R) + r) + 1] = rstd;
            }
            lds_barrier();
        }
        STAMP(sti++);
        if (yq)
            ln_full(T1, S1, T1, S1, HW, nk, mu, rstd, lp, P + o[4], P + o[5]);
        else if (SA(nwin) == 1)
            ln_apply(T1, S1, T1, S1, HW, SA(win_off)[0], SA(win_len)[0], nk, mu, rstd, ln ? P + o[4] : nullptr,
                     ln ? P + o[5] : nullptr, ln);
        else
            ln_windows(T1, S1, HW, nk, SA(nwin), SA(win_off), SA(win_len), mu, rstd, ln ? P + o[4] : nullptr,
                       ln ? P + o[5] : nullptr, ln);
        STAMP(sti++);
        if (tq) lnp_load(lp, P + o[6], P + o[7], HW * gc / 4);
        // grouped dilated branches -> T2[:, out_off : out_off + cout] (+ LN3 stats over all of them)
        // every branch's packed image (contiguous in aux: weights + bias per branch) and tap / quad
        // table staged at once: the branches run back to back without barriers between them (they
        // read T1 and write disjoint T2 slices), each wave merging its LN3 partials across them
        if (r == 0) {   // the same for every residual block (conv_out builds its own after the loop)
            int kto = 0;
            for (int bi = 0; bi < SA(nbr); bi++) {
                const LdsConv& cv = SA(gcv)[bi];
                conv3_table(cv, KT + kto, SA(br_cin)[bi], SA(br_cin_off)[bi], SA(br_dil)[bi]);
                kto += ktab_len(cv);
            }
        }
        STAMP(sti++);
        wpf_store(pf, WL, X + o[10]);
        STAMP(sti++);
        lds_barrier();   // LN2 applied, slots read, branch images and tables complete
        lst_reset(st);
        wpf_load(pf, X + o[8], wb(SA(cb), nk));
        STAMP(sti++);
        {
            int kto = 0;
            auto run_br = [&](int bi) {
                const LdsConv& cv = SA(gcv)[bi];
                const float* wbr = WL + (o[10 + 2 * bi] - o[10]);
                conv3_run<MAXNR, (SID >= 0)>(cv, T1, S1, H, W, wbr, KT + kto, T2 + SA(br_out_off)[bi], S2,
                                             SA(br_cout)[bi], WL + (o[11 + 2 * bi] - o[10]), st, ln, ZQ,
                                             KSplit{ksb, bi & 1},
                                             KTap{SA(br_cin)[bi], SA(br_cin_off)[bi], SA(br_dil)[bi]});
                kto += ktab_len(cv);
            };
            if constexpr (SID >= 0) {   // unrolled: every branch's format, extents and offsets constant
#pragma unroll
                for (int bi = 0; bi < kNetShapes[SID >= 0 ? SID : 0].nbr; bi++) run_br(bi);
            } else {
                for (int bi = 0; bi < SA(nbr); bi++) run_br(bi);
            }
        }
        if (ln) lst_flush(st, slots);
        STAMP(sti++);
        lds_barrier();
        STAMP(sti++);
        // LN3(LReLU(t2)) in place, conv_b (1x1 gc->nk) + shortcut -> Y (+ LN stats of Y)
        if (ln) lst_final(slots, mu, rstd);
        if (sv != nullptr) {   // raw t2_r and LN3_r, before LN3 is applied in place
            save_tensor(T2, S2, HW, gc, sv + a.save_t2 + (size_t)r * HW * gc);
            if (threadIdx.x == 0) {
                sv[a.save_st + 2 * (2 * SA(R) + r)] = mu;
                sv[a.save_st + 2 * (2 * SA(R) + r) + 1] = rstd;
            }
            lds_barrier();
        }
        STAMP(sti++);
        if (tq)
            ln_full(T2, S2, T2, S2, HW, gc, mu, rstd, lp, P + o[6], P + o[7]);
        else
            ln_apply(T2, S2, T2, S2, HW, 0, gc, gc, mu, rstd, ln ? P + o[6] : nullptr, ln ? P + o[7] : nullptr, ln);
        STAMP(sti++);
        wpf_store(pf, WL, X + o[8]);
        STAMP(sti++);
        lds_barrier();
        lst_reset(st);
        if (r + 1 < SA(R))
            wpf_load(pf, X + rbo(r + 1)[2], wb(SA(ca), nk));
        else
            wpf_load(pf, X + oend[2], wb(SA(co), SA(dc2)));
        if (yq)
            lnp_load(lp, P + (r + 1 < SA(R) ? rbo(r + 1)[0] : oend[0]), P + (r + 1 < SA(R) ? rbo(r + 1)[1] : oend[1]),
                     HW * nk / 4);
        STAMP(sti++);
        conv1_any<MAXNR>(T2, S2, gc, HW, WL, Y, SY, nk, WL + SA(cb).size, true, st, ln, ks0);
        if (ln) lst_flush(st, slots);
        STAMP(sti++);
        lds_barrier();
        STAMP(sti++);
    }
    // LN_out(LReLU(y)) in place, conv_out (3x3 nk -> dc2) -> global
    {
        const int* o = oend;
        if (ln) lst_final(slots, mu, rstd);
        if (sv != nullptr) {   // y_R and LN_out, before LN_out is applied in place
            save_tensor(Y, SY, HW, nk, sv + (size_t)SA(R) * HW * nk);
            if (threadIdx.x == 0) {
                sv[a.save_st + 6 * SA(R)] = mu;
                sv[a.save_st + 6 * SA(R) + 1] = rstd;
            }
            lds_barrier();
        }
        if (yq)
            ln_full(Y, SY, Y, SY, HW, nk, mu, rstd, lp, P + o[0], P + o[1]);
        else
            ln_apply(Y, SY, Y, SY, HW, 0, nk, nk, mu, rstd, ln ? P + o[0] : nullptr, ln ? P + o[1] : nullptr, ln);
        STAMP(sti++);
        float* dst = a.so[net] + (size_t)img * HW * SA(dc2);
        const float* bias = WL + SA(co).size;
        if (SA(co).fmt == PK_TAP) {
            // tap-decomposed: C[p][(tap, o)] = sum_c y[p][c] W[tap][c][o] (1x1 GEMM, scratch over T1..T2),
            // out[p][o] = b[o] + sum_tap C[p + off(tap)][(tap, o)]
            const int ncol = 9 * SA(dc2);
            const int co_nr = (ncol + 15) / 16;
            const bool vq = (SA(dc2) & 3) == 0;   // quad-shaped output: 16-byte tap-sum reads
            const int CS = 16 * co_nr + (vq ? 4 : 1);
            float* C = T1;
            wpf_store(pf, WL, X + o[2]);
            lds_barrier();
            // in chunks of CB 16-column blocks (the narrow instantiation computes at most two at once)
            constexpr int CB = MAXNR >= 5 ? 5 : 2;
            STAMP(sti++);
            for (int nb = 0; nb < co_nr; nb += CB)
                conv1_any<MAXNR>(Y, SY, nk, HW, WL, C + 16 * nb, CS, min(16 * CB, ncol - 16 * nb), nullptr, false, st,
                                 false, KSplit{ksb, (nb / CB) & 1}, 16 * co_nr, nb);
            STAMP(sti++);
            lds_barrier();
            STAMP(sti++);
            if (vq) {
                // one output quad per item: 9 tap quads issued together (outside the image: ZQ)
                const int nq = SA(dc2) >> 2, n = HW * nq;
                for (int e = threadIdx.x; e < n; e += NT) {
                    const int p = e / nq, oq = (e - p * nq) << 2;
                    const int pr = p / W, pc = p - pr * W;
                    f4 t[9];
#pragma unroll
                    for (int k = 0; k < 9; k++) {
                        const int sr = pr + k / 3 - 1, sc = pc + k % 3 - 1;
                        const bool ok = (unsigned)sr < (unsigned)H && (unsigned)sc < (unsigned)W;
                        t[k] = *reinterpret_cast<const f4*>(ok ? C + (sr * W + sc) * CS + k * SA(dc2) + oq : ZQ);
                    }
                    f4 acc = *reinterpret_cast<const f4*>(bias + oq);
#pragma unroll
                    for (int k = 0; k < 9; k++) acc += t[k];
                    *reinterpret_cast<f4*>(dst + p * SA(dc2) + oq) = acc;
                }
            } else {
                const int n = HW * SA(dc2);
                for (int e = threadIdx.x; e < n; e += NT) {
                    const int p = e / SA(dc2), oc = e - p * SA(dc2);
                    const int pr = p / W, pc = p - pr * W;
                    float acc = bias[oc];
#pragma unroll
                    for (int kh = 0; kh < 3; kh++) {
                        const int sr = pr + kh - 1;
                        if (sr < 0 || sr >= H) continue;
#pragma unroll
                        for (int kw = 0; kw < 3; kw++) {
                            const int sc = pc + kw - 1;
                            if (sc < 0 || sc >= W) continue;
                            acc += C[(sr * W + sc) * CS + (kh * 3 + kw) * SA(dc2) + oc];
                        }
                    }
                    dst[e] = acc;
                }
            }
        } else {
            conv3_table(SA(co), KT, nk, 0, 1);
            wpf_store(pf, WL, X + o[2]);
            lds_barrier();
            conv3_run<MAXNR>(SA(co), Y, SY, H, W, WL, KT, T2, S2, SA(dc2), bias, st, false, ZQ, ks0);
            lds_barrier();
            const int n = HW * SA(dc2);
            for (int e = threadIdx.x; e < n; e += NT) {
                const int p = e / SA(dc2), c = e - p * SA(dc2);
                dst[e] = T2[p * S2 + c];
            }
        }
    }
    if (a.pend.on != 0 && a.pend.comp == 0) {
        // the deferred coupling's v_k and log-det partials (after conv_out: its loads and stores
        // then add to the kernel's tail instead of delaying conv_in)
        const CoupPend& q = a.pend;
        const int n_img = SA(H) * SA(W) * SA(D);
        const float* ub = q.u + (size_t)img * n_img;
        const size_t sb = (size_t)img * q.hc * q.wc * q.dc2;
        const float w = *q.tanh_w;
        auto coupled = [&](int pos, float& s) {
            const int ci = pend_index(q, pos, SA(W), SA(D));
            const float x = ub[pos];
            if (ci < 0) return x;
            s = w * cpl_tanh(q.s_pre[sb + ci]);
            return cpl_law(s, x, q.t[sb + ci], q.dir);
        };
        const bool split = q.np >= 2;
        const int e0 = split && net == 1 ? n_img / 2 : 0, e1 = split && net == 0 ? n_img / 2 : n_img;
        float lsum = 0.f;
        if (!split && net == 1) {
            // (one slot per image: net A's workgroup writes the whole v_k)
        } else {
            float* vb = q.v + (size_t)img * n_img;
            for (int e = e0 + (int)threadIdx.x; e < e1; e += NT) {
                float s = 0.f;
                vb[e] = coupled(e, s);
                lsum += s;
            }
        }
        lds_barrier();   // (lst_final's reads of the LN slots are done)
        double* lsl = reinterpret_cast<double*>(slots);   // NW doubles (LN slots: free after conv_out)
        const double ws = wave_sum((double)lsum);
        if ((threadIdx.x & 63) == 0) lsl[threadIdx.x >> 6] = ws;
        lds_barrier();
        if (threadIdx.x == 0 && (split || net == 0) && q.ld_part != nullptr) {   // (the inverse has none)
            double t = 0.0;
            for (int i = 0; i < NW; i++) t += lsl[i];
            double* dst = q.ld_part + (size_t)img * q.np;
            dst[net] = t;
            if (net == 0)
                for (int j = 2; j < q.np; j++) dst[j] = 0.0;
        }
        lds_barrier();
    }
    STAMP(sti++);
    if (STAMPS && threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) {
        g_stamps[0] = rt0;
        g_stamps[1] = (long long)__builtin_amdgcn_s_memrealtime();
        for (int i = 0; i < sti && i < 128; i++) g_cycles[i] = stamp_lds[i];
        g_stamps[255] = sti;
    }
}

// instantiation flags of table entry S: narrow (<= 2 output blocks) and K-split
template <int S>
constexpr bool shape_narrow() { return kNetShapeWords[S][NETSHAPE_W1 + NETSHAPE_W2 - 1] <= 2; }
template <int S>
constexpr bool shape_ks() { return !CNF_NETLDS_NOKS && kNetShapeWords[S][NETSHAPE_W1 + NETSHAPE_W2 - 2] != 0; }

template <int S>
bool launch_shape(int sid, const NetLdsArgs& a, dim3 grid, dim3 block, int lds, hipStream_t st, bool stamps) {
    if constexpr (S < CNF_NETLDS_NSHAPES) {
        if (sid == S) {
            if (stamps) {
                NetLdsArgs b = a;
                b.stamp_off = (lds + 15) & ~15;
                CNF_LAUNCH((k_net_lds<true, shape_narrow<S>() ? 2 : 5, shape_ks<S>(), S>), grid, block,
                                   b.stamp_off + 1024, st, b);
            } else {
                CNF_LAUNCH((k_net_lds<false, shape_narrow<S>() ? 2 : 5, shape_ks<S>(), S>), grid, block, lds, st, a);
            }
            return true;
        }
        return launch_shape<S + 1>(sid, a, grid, block, lds, st, stamps);
    }
    return false;
}

int netlds_num_shapes() { return CNF_NETLDS_NSHAPES; }

void launch_net_lds(const NetLdsArgs& a, int B, int lds, hipStream_t st) {
#ifdef CNF_DIAG
    static const bool stamps = [] {   // diagnostic builds: phase stamps (profiles/diag/diag_stamps.py)
        const char* e = std::getenv("CNF_STAMPS");
        return e && std::atoi(e) != 0;
    }();
#else
    constexpr bool stamps = false;
#endif
    const bool generic = (opts().generic & 9) != 0;   // debug option GENERIC bit 1 (all) or 8 (k_net_lds)
    const bool narrow = a.maxnr <= 2;
    const bool ks = a.off_ks != 0;
    const dim3 grid(B, 2), block(NT);
    if (!generic) {
        int w[NETSHAPE_WORDS];
        netshape_words(a, w);
        for (int sid = 0; sid < CNF_NETLDS_NSHAPES; sid++) {
            bool eq = true;
            for (int i = 0; i < NETSHAPE_WORDS && eq; i++) eq = w[i] == kNetShapeWords[sid][i];
            if (eq && launch_shape<0>(sid, a, grid, block, lds, st, stamps)) return;
        }
    }
    if (stamps) {
        NetLdsArgs b = a;
        b.stamp_off = (lds + 15) & ~15;
        const int l2 = b.stamp_off + 1024;
        if (narrow && ks)
            CNF_LAUNCH((k_net_lds<true, 2, true, -1>), grid, block, l2, st, b);
        else if (narrow)
            CNF_LAUNCH((k_net_lds<true, 2, false, -1>), grid, block, l2, st, b);
        else
            CNF_LAUNCH((k_net_lds<true, 5, false, -1>), grid, block, l2, st, b);
        return;
    }
    if (narrow && ks) {
        CNF_LAUNCH((k_net_lds<false, 2, true, -1>), grid, block, lds, st, a);
    } else if (narrow) {
        CNF_LAUNCH((k_net_lds<false, 2, false, -1>), grid, block, lds, st, a);
    } else {
        CNF_LAUNCH((k_net_lds<false, 5, false, -1>), grid, block, lds, st, a);
    }
}

int read_cycles(long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_cycles), sizeof(long long) * (n > 256 ? 256 : n)) == hipSuccess ? 0 : -1;
}

int read_stamps(long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamps), sizeof(long long) * (n > 256 ? 256 : n)) == hipSuccess ? 0 : -1;
}

}  // namespace cnf
