// cnf_device.h — device helpers shared by the conv kernels (cnf_kernels.hip, cnf_stream.hip).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

#include "cnf_kernels.h"

namespace cnf {

typedef float f4 __attribute__((ext_vector_type(4)));

// Workgroup barrier for LDS hand-offs only: waits for this wave's LDS operations, then s_barrier.
// Unlike __syncthreads() it does not drain outstanding global loads (vmcnt), so register prefetches
// issued before a barrier (next conv's weights, LN gamma/beta) stay in flight across it. Global
// data never passes between the waves of a workgroup through these barriers.
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// LeakyReLU(alpha = 0.3): max(x, 0.3 x) == (x >= 0 ? x : 0.3 x) for every finite x, in 2 VALU ops:
// fmaxf of a loaded x costs a third, the IEEE-mode canonicalisation v_max_f32 x, x, which this form
// leaves out (it only quiets signalling NaNs). Measured: conv_b 30.6 -> 29.3 us, the cfg2 forward
// 1.473 -> 1.447 ms
__device__ __forceinline__ float lrelu(float x) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(x), "v"(LRELU_ALPHA * x));
    return r;
}

// n / d for n >= 0, n * d < 2^32 as one multiply-high: m = udiv_magic(d) = ceil(2^32 / d) (0 for d == 1)
// — the runtime-shape training kernels divide flat indices per element, and the compiler's generic
// 32-bit division is ~30 VALU instructions (it made those kernels VALU-issue-bound)
__host__ __device__ __forceinline__ uint32_t udiv_magic(uint32_t d) { return d <= 1 ? 0u : 0xFFFFFFFFu / d + 1u; }
__device__ __forceinline__ int udiv(int n, uint32_t m) { return m == 0 ? n : (int)__umulhi((uint32_t)n, m); }

// tanh and exp of the affine coupling law (s = w * tanh(A), exp(s): conv_cINN_make_model.py:1198-1205,
// 1215-1253) on the hardware exp (v_exp_f32): an odd Taylor polynomial below |x| = 1/4 (truncation
// < 1e-8 relative), 1 - 2 / (e^{2|x|} + 1) above (< 1e-6 relative). k_coupling, the deferred coupling
// in k_net_lds and the coupling backward all use these, so their results agree bit for bit.
__device__ __forceinline__ float cpl_tanh(float x) {
    const float ax = fabsf(x);
    if (ax < 0.25f) {
        const float x2 = x * x;
        const float p = fmaf(x2, fmaf(x2, fmaf(x2, fmaf(x2, 62.f / 2835.f, -17.f / 315.f), 2.f / 15.f), -1.f / 3.f), 1.f);
        return x * p;
    }
    const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(__expf(2.f * ax) + 1.f);   // e^{2|x|} = inf -> 1
    return copysignf(t, x);
}
__device__ __forceinline__ float cpl_exp(float s) { return __expf(s); }
// the affine law on one transformed element (k_coupling, and the deferred law in k_net_lds / k_map2:
// one expression, so the fused schedules equal the layer-by-layer API bit for bit)
// dir > 0: v2 = exp(s) u2 + t (:1215-1233); dir < 0: u2 = reciprocal(exp(s)) (v2 - t) (:1235-1253)
__device__ __forceinline__ float cpl_law(float s, float x, float t, int dir) {
    return dir > 0 ? fmaf(cpl_exp(s), x, t) : (1.0f / cpl_exp(s)) * (x - t);
}

// compressed index (p * dc2 + c) in layer k's transformed half of element pos of u_k, or -1 when pos
// lies in its conditioning half: the inverse of mask_pos_ for the complement mask q.mask_c
__device__ __forceinline__ int pend_index(const CoupPend& q, int pos, int W, int D) {
    const int pix = pos / D, ch = pos - pix * D;
    const int y = pix / W, x = pix - y * W;
    if (q.mask_c < 2) {   // checkerboard: c0 -> (even, even) / (even, odd), c1 -> (odd, odd) / (odd, even)
        const int half = y & 1;
        if (((x & 1) == half) != (q.mask_c == 0)) return -1;
        return ((y >> 1) * q.wc + (x >> 1)) * q.dc2 + half * D + ch;
    }
    if ((ch & 1) != (q.mask_c == 3 ? 1 : 0)) return -1;   // channels 0::2 / 1::2
    return pix * q.dc2 + (ch >> 1);
}


// Philox4x32-10 (Salmon et al. 2011): counter (c0..c3), key (k0, k1), 10 rounds in place
__device__ __forceinline__ void philox(uint32_t c[4], uint32_t k0, uint32_t k1) {
#pragma unroll
    for (int r = 0; r < 10; r++) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c[0], p1 = (uint64_t)0xCD9E8D57u * c[2];
        const uint32_t n0 = (uint32_t)(p1 >> 32) ^ c[1] ^ k0, n1 = (uint32_t)p1;
        const uint32_t n2 = (uint32_t)(p0 >> 32) ^ c[3] ^ k1, n3 = (uint32_t)p0;
        c[0] = n0;
        c[1] = n1;
        c[2] = n2;
        c[3] = n3;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
}
// instance_noise (conv_cINN_base_functions.py:635-654) of element g of the stream (g = offset + flat
// index): alpha x + (1 - alpha) z, z ~ N(0, 1) by Box-Muller on the Philox words of counter g / 4
// (4 normals per counter value, element g taking normal g % 4). One expression for k_noise and the
// forward's fused first-layer gather (cnf_flow_forward_noise), so the two agree bit for bit.
// x_or_null == false: renew_noise (:660-676), z alone.
__device__ __forceinline__ float instance_noise_value(float x, bool has_x, float alpha, uint64_t seed, uint64_t g) {
    uint32_t c[4] = {(uint32_t)(g >> 2), (uint32_t)(g >> 34), 0u, 0u};
    philox(c, (uint32_t)seed, (uint32_t)(seed >> 32));
    const int w = (int)(g & 3);
    const int pair = w >> 1;
    // uniform in (0, 1] and [0, 1)
    const float u1 = ((float)(c[2 * pair] >> 8) + 1.f) * (1.f / 16777216.f);
    const float u2 = (float)(c[2 * pair + 1] >> 8) * (1.f / 16777216.f);
    const float rad = sqrtf(-2.f * logf(u1));
    const float th = 6.283185307179586f * u2;
    const float z = (w & 1) ? rad * sinf(th) : rad * cosf(th);
    return has_x ? fmaf(alpha, x, (1.f - alpha) * z) : z;
}

// the reference's logit preprocess of x (preprocess_dataset_class(LOGITS=True), :174-231):
// v -> (logit(a + (1 - a) b v) - logit(a)) / (logit(1 - a) - logit(a)); k_logit and the fused
// input preparation share this expression
__device__ __forceinline__ float logit_value(float v, const LogitK& k) {
    const float e = fmaf(k.c1, v, k.a);
    return (logf(e / (1.f - e)) - k.lo) / k.span;
}
// InputPrepArgs (cnf_kernels.h) of element g of the batch stream, channel ch: cnf_flow_forward_noise's
// fused gather and its k_prep fallback use this one expression, bit for bit the k_logit + k_noise passes
__device__ __forceinline__ float input_prep_value(float x, int ch, const InputPrepArgs& q, uint64_t g) {
    if (q.logit && ch < q.x_d) x = logit_value(x, q.lk);
    return instance_noise_value(x, true, q.alpha, q.seed, g);
}

// Wave-wide fp32 sum by DPP lane moves (quad_perm, row_shr, row_bcast: a few cycles each instead
// of an LDS-routed ds_bpermute per step); lane 63 ends with the total, broadcast by readlane.
// Out-of-range source lanes read 0 (update_dpp with old = 0). Fixed order: bitwise reproducible.
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
    return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
__device__ __forceinline__ float wave_sum_f(float v) {
    v += dpp_f<0xb1>(v);    // quad_perm [1,0,3,2]
    v += dpp_f<0x4e>(v);    // quad_perm [2,3,0,1]
    v += dpp_f<0x114>(v);   // row_shr:4
    v += dpp_f<0x118>(v);   // row_shr:8   -> lane 15 of each row holds the row sum
    v += dpp_f<0x142>(v);   // row_bcast:15
    v += dpp_f<0x143>(v);   // row_bcast:31 -> lane 63 holds the wave sum
    return __builtin_bit_cast(float, __builtin_amdgcn_readlane(__builtin_bit_cast(int, v), 63));
}

// raw buffer resource over [base, base + bytes): loads beyond the range return 0, stores beyond it
// are dropped — used for branch-free masking (offset BUF_OOB) and 32-bit offsets.
constexpr uint32_t BUF_OOB = 0x80000000u;
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, uint32_t bytes) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)bytes, 0x00020000);
}
__device__ __forceinline__ f4 buf_load4(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(f4, __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0));
}
__device__ __forceinline__ float buf_load1(__amdgpu_buffer_rsrc_t r, uint32_t off) {
    return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(r, off, 0, 0));
}
__device__ __forceinline__ void buf_store1(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, v), r, off, 0, 0);
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

__device__ __forceinline__ bool stored(const ConvProb& P, int ch) {
    return ((ch < 32 ? (P.st_mask_lo >> ch) : (P.st_mask_hi >> (ch - 32))) & 1u) != 0u;
}

// LN statistics of a conv output, produced in the conv's epilogue (no extra pass, no barrier):
// each wave writes the partial (K, S1, S2, n) of the LeakyReLU'd values its lanes hold — fp32 sums
// shifted by a wave-uniform sample value K (readfirstlane), so sum (x-K)^2 does not cancel — as
// one 16-byte store by lane 0 (DPP reductions, no division, no fp64).
template <int N>
__device__ __forceinline__ void ln_partial(const float (&vals)[N], const bool (&valid)[N], float* __restrict__ dst) {
#ifdef CNF_ABL_NOPART
    return;
#endif
    const float K = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, vals[0])));
    float s1 = 0.f, s2 = 0.f, c = 0.f;
#pragma unroll
    for (int i = 0; i < N; i++) {
        const float d = valid[i] ? vals[i] - K : 0.f;
        s1 += d;
        s2 = fmaf(d, d, s2);
        c += valid[i] ? 1.f : 0.f;
    }
    s1 = wave_sum_f(s1);
    s2 = wave_sum_f(s2);
    c = wave_sum_f(c);
    if ((threadIdx.x & 63) == 0) *reinterpret_cast<f4*>(dst) = f4{K, s1, s2, c};
}

// Streaming form of ln_partial for epilogues that produce their values in several steps: lanes
// accumulate shifted fp32 sums; write() reduces over the wave and stores (K, S1, S2, n).
struct LnAcc {
    float K, s1, s2, c;
    __device__ __forceinline__ void reset() { K = s1 = s2 = c = 0.f; }
    // shift = lane 0's value (call in wave-uniform control flow, before the first add)
    __device__ __forceinline__ void set_shift(float lrelu_v) {
        K = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, lrelu_v)));
    }
    __device__ __forceinline__ void add(float lrelu_v, bool valid) {
        const float d = valid ? lrelu_v - K : 0.f;
        s1 += d;
        s2 = fmaf(d, d, s2);
        c += valid ? 1.f : 0.f;
    }
    __device__ __forceinline__ void write(float* __restrict__ dst) const {
#ifdef CNF_ABL_NOPART
        return;
#endif
        const float S1 = wave_sum_f(s1), S2 = wave_sum_f(s2), C = wave_sum_f(c);
        if ((threadIdx.x & 63) == 0) *reinterpret_cast<f4*>(dst) = f4{K, S1, S2, C};
    }
};

// (mean, rstd) of the input LayerNorm of image img from the producer's partials, merged by every
// wave on its own (no barrier); identity without LN. Each lane folds its partials (Chan merge when
// it holds more than one), then the wave merges per-lane (n, mean, M2) in the parallel-axis form
// (N = sum n, mean = sum n m / N, M2 = sum M2 + n (m - mean)^2) with DPP sums: fixed order, fp32.
// one partial (K, S1, S2, n) folded into a lane's running (n, mean, M2)
__device__ __forceinline__ void ln_fold(const f4 v, float& n, float& m, float& M2) {
    if (v[3] > 0.f) {
        const float r = v[1] * __builtin_amdgcn_rcpf(v[3]);
        const float mi = v[0] + r, M2i = fmaxf(fmaf(-v[1], r, v[2]), 0.f);
        const float nn = n + v[3], dl = mi - m, f = v[3] * __builtin_amdgcn_rcpf(nn);
        m = fmaf(dl, f, m);
        M2 = M2 + M2i + dl * dl * n * f;
        n = nn;
    }
}
// wave merge of the lanes' (n, mean, M2) -> (mean, rstd)
__device__ __forceinline__ void ln_wave_final(float n, float m, float M2, float& mu, float& rstd) {
    const float N = wave_sum_f(n);
    const float iN = __builtin_amdgcn_rcpf(N);
    const float mean = wave_sum_f(n * m) * iN;
    const float d = m - mean;
    const float M = wave_sum_f(fmaf(n * d, d, M2));
    mu = mean;
    rstd = __builtin_amdgcn_rsqf(fmaf(M, iN, LN_EPS));
}
// a lane's first partial: its (n, mean, M2) directly (no merge with the empty state, whose
// n * rcp(n) need not be exactly 1)
__device__ __forceinline__ void ln_fold_first(const f4 v, float& n, float& m, float& M2) {
    n = 0.f;
    m = 0.f;
    M2 = 0.f;
    if (v[3] > 0.f) {
        const float r = v[1] * __builtin_amdgcn_rcpf(v[3]);
        m = v[0] + r;
        M2 = fmaxf(fmaf(-v[1], r, v[2]), 0.f);
        n = v[3];
    }
}
// Split form of in_ln for prologues: in_ln_fetch issues the lane's first LN_FETCH partial-slot loads
// early (slots lane, lane + 64, ...: with the prologue's other global loads, so they share one memory
// round trip), in_ln_finish folds them and any further slots. in_ln is in_ln_fetch + in_ln_finish, so
// an image's (mean, rstd) are the same bits whichever form computes them: the form depends on the
// image's position in its workgroup's image set, i.e. on the batch size (the round-4 batch
// dependence: ln_fold of the first slot into the empty state and this path contracted differently).
// Producers of up to 64 * LN_FETCH slots per image (the 64x64 layers' k_gc groups) need no k_ln_merge
// (LN_FETCH: cnf_kernels.h).
struct LnSlots {
    f4 v[LN_FETCH];
};
__device__ __forceinline__ LnSlots in_ln_fetch(const ConvProb& P, int img) {
    const int lane = threadIdx.x & 63;
    LnSlots s;
#pragma unroll
    for (int k = 0; k < LN_FETCH; k++) {
        const int i = lane + 64 * k;
        s.v[k] = P.in_part != nullptr && i < P.in_nparts
                     ? *reinterpret_cast<const f4*>(P.in_part + ((size_t)img * P.part_stride + i) * LNP)
                     : f4{0.f, 0.f, 0.f, 0.f};
    }
    return s;
}
__device__ __forceinline__ void in_ln_finish(const ConvProb& P, int img, const LnSlots& s, float& mu, float& rstd) {
    mu = 0.f;
    rstd = 1.f;
    if (P.in_part == nullptr) return;
#ifdef CNF_ABL_NOINLN
    return;
#endif
    float n, m, M2;
    ln_fold_first(s.v[0], n, m, M2);
#pragma unroll
    for (int k = 1; k < LN_FETCH; k++) ln_fold(s.v[k], n, m, M2);   // (empty slots: v[3] == 0, skipped)
    const float* __restrict__ q = P.in_part + (size_t)img * P.part_stride * LNP;
    for (int i = (threadIdx.x & 63) + 64 * LN_FETCH; i < P.in_nparts; i += 64) {
        const f4 w = *reinterpret_cast<const f4*>(q + (size_t)LNP * i);
        ln_fold(w, n, m, M2);
    }
    ln_wave_final(n, m, M2, mu, rstd);
}
__device__ __forceinline__ void in_ln(const ConvProb& P, int img, float& mu, float& rstd) {
    in_ln_finish(P, img, in_ln_fetch(P, img), mu, rstd);
}

// Copy n floats (n % 4 == 0, both 16-byte aligned) global -> LDS; 8 float4 loads in flight per thread.
template <int NTH>
__device__ __forceinline__ void copy_to_lds(const float* __restrict__ src, float* dst, int n) {
    const int n4 = n >> 2;
    const f4* s4 = reinterpret_cast<const f4*>(src);
    f4* d4 = reinterpret_cast<f4*>(dst);
    for (int base = 0; base < n4; base += NTH * 8) {
        f4 v[8];
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int i = base + u * NTH + (int)threadIdx.x;
            v[u] = i < n4 ? s4[i] : f4{0.f, 0.f, 0.f, 0.f};
        }
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int i = base + u * NTH + (int)threadIdx.x;
            if (i < n4) d4[i] = v[u];
        }
    }
}

// ---------------------------------------------------------------------------------------------
// fp32 contractions on the bf16 matrix cores (bf16x6). Every fp32 operand x is split exactly into
// three bf16 terms, x = h + m + l: h = bf16(x), m = bf16(x - h), l = x - h - m (both differences are
// exact in fp32: they are the low bits of x; l has at most 8 significant bits, so it is a bf16). With
// |m| <= 2^-8 |x| and |l| <= 2^-16 |x|, a product x w is h H + h M + m H + h L + l H + m M (six bf16
// MFMA products, each exact in fp32) up to the dropped m L + l M + l L: at most 2^-23 |x w| (one fp32
// ulp), 2^-26 on average, the size of the rounding of one fp32 product. The sums accumulate in fp32 in
// the MFMA. One 16x16x32 bf16 MFMA takes
// 16 cycles against 32 for the 16x16x4 fp32 one: six of them per 32-deep K step are 0.375x the fp32
// MFMA time of the same contraction.
// ---------------------------------------------------------------------------------------------
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));
struct Split8 {
    bf16x8 h, m, l;
};
__device__ __forceinline__ void split3(float x, __bf16& h, __bf16& m, __bf16& l) {
    h = (__bf16)x;
    const float r = x - (float)h;
    m = (__bf16)r;
    l = (__bf16)(r - (float)m);
}
// the lane's 8 consecutive K elements (a: k 0..3, b: k 4..7) as the three bf16 fragments
__device__ __forceinline__ Split8 split8(const f4& a, const f4& b) {
    Split8 s;
#pragma unroll
    for (int j = 0; j < 4; j++) {
        __bf16 h, m, l;
        split3(a[j], h, m, l);
        s.h[j] = h;
        s.m[j] = m;
        s.l[j] = l;
        split3(b[j], h, m, l);
        s.h[4 + j] = h;
        s.m[4 + j] = m;
        s.l[4 + j] = l;
    }
    return s;
}
__device__ __forceinline__ void split4(const f4& a, bf16x4& h, bf16x4& m, bf16x4& l) {
#pragma unroll
    for (int j = 0; j < 4; j++) {
        __bf16 x, y, z;
        split3(a[j], x, y, z);
        h[j] = x;
        m[j] = y;
        l[j] = z;
    }
}
// acc += A . B over one 32-deep K step (16x16x32, A rows / B columns per the lane maps of the bf16
// MFMA), A = a.h + a.m + a.l, B = bh + bm + bl; the small products first
__device__ __forceinline__ f4 mfma_x6(const bf16x8& ah, const bf16x8& am, const bf16x8& al, const bf16x8& bh,
                                      const bf16x8& bm, const bf16x8& bl, f4 acc) {
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(al, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bl, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(am, bh, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bm, acc, 0, 0, 0);
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah, bh, acc, 0, 0, 0);
    return acc;
}

// masks (conv_cINN_make_model.py:720-759, 896-1071)
// position in u (per-image element index) of element (compressed pixel p, channel c) of the
// compressed half selected by mask m.
__device__ __forceinline__ int mask_pos(int m, int p, int c, int wc, int W, int D) {
    const int pr = p / wc, pc = p - pr * wc;
    if (m < 2) {
        const int half = c >= D ? 1 : 0;
        const int ch = c - half * D;
        // mask 0: c0 -> (even, even), c1 -> (odd, odd); mask 1: c0 -> (even, odd), c1 -> (odd, even)
        const int dr = half;
        const int dc = (m == 0) ? half : 1 - half;
        return ((2 * pr + dr) * W + (2 * pc + dc)) * D + ch;
    }
    const int ch = (m == 2) ? 2 * c : 2 * c + 1;
    return (pr * W + pc) * D + ch;
}

}  // namespace cnf
