// cnf_stream.hip — image-looping streamed convolutions for coupling layers whose s,t-net
// activations do not fit one CU's LDS (k_net_lds covers the rest).
//
//   k_pw   1x1 convolution (conv_a / conv_b of dilated_residual_block,
//          conv_cINN_base_functions.py:561-565, 609-613) with LeakyReLU -> per-image LayerNorm
//          (per-element gamma/beta, :330-362) applied on load, bias + residual in the epilogue
//          and the per-wave LN partials of LeakyReLU(out) for the next LayerNorm.
//
// Work decomposition: a workgroup owns one 64-pixel tile (16 pixels per wave) of MI images. The
// LN gamma/beta of the tile are image-independent, so one register copy serves all MI images.
#include <stdexcept>

#include "cnf_device.h"

namespace cnf {

constexpr int PW_TILE = 64;         // pixels per workgroup tile
constexpr int PW_LDS_STAT = 256;    // byte offset of the per-image (mean, rstd) table

// One workgroup = one 64-pixel tile (16 pixels per wave) x MI images, all in flight at once:
// every activation load of the workgroup is issued up front (one memory round trip), the LN
// gamma/beta registers of the tile serve all MI images, and each B-quad LDS read feeds 4*MI
// MFMAs. No loop-carried waits: latency is covered by the MI*G float4 loads each lane has in flight.
template <int NR, int GM, int MI, bool LN, bool RES>
__global__ __launch_bounds__(256, 2) void k_pw(ConvArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const ConvProb P = a.p[blockIdx.y];
    const int HW = a.H * a.W;
    const int tile = blockIdx.x % a.tiles_per_img;
    const int img0 = (blockIdx.x / a.tiles_per_img) * MI;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int i16 = lane & 15, kq = lane >> 4;
    const int cin = P.cin, G = (cin + 15) >> 4, cout = P.cout;
    constexpr int NSJ = 16 * NR;
    float* lw = reinterpret_cast<float*>(smem + P.lds_w_off);
    float* lstat = reinterpret_cast<float*>(smem + PW_LDS_STAT);
    // buffer resources: out-of-range offsets (BUF_OOB) load 0 / drop the store
    const uint32_t in_img = (uint32_t)HW * P.in_cs * 4u, out_img = (uint32_t)HW * P.out_cs * 4u;
    const auto rin = buf_rsrc(P.in, (uint32_t)a.B * in_img);
    const auto rout = buf_rsrc(P.out, (uint32_t)a.B * out_img);

    // A operand: lane (i16, kq) feeds pixel pa, channels 16g + 4kq + s at k-step s of group g
    const int pa = tile * PW_TILE + wave * 16 + i16;
    const bool pav = pa < HW;
    const uint32_t aoff = ((uint32_t)pa * P.in_cs + P.in_off + 4 * kq) * 4u;
    uint32_t goff[GM];   // byte offset of group g inside one image, BUF_OOB when masked
#pragma unroll
    for (int g = 0; g < GM; g++) goff[g] = (pav && g < G && 16 * g + 4 * kq < cin) ? aoff + 64u * g : BUF_OOB;
    f4 x[MI][GM];
#pragma unroll
    for (int m = 0; m < MI; m++) {
        const uint32_t ib = img0 + m < a.B ? (uint32_t)(img0 + m) * in_img : BUF_OOB;
#pragma unroll
        for (int g = 0; g < GM; g++) x[m][g] = buf_load4(rin, goff[g] == BUF_OOB ? BUF_OOB : ib + goff[g]);
    }
    f4 gm[GM], bt[GM];
    if (LN) {
        const auto rg = buf_rsrc(P.gamma, in_img), rb = buf_rsrc(P.beta, in_img);
#pragma unroll
        for (int g = 0; g < GM; g++) {
            gm[g] = buf_load4(rg, goff[g]);   // 0 where masked: the normalised value is then exactly 0
            bt[g] = buf_load4(rb, goff[g]);
        }
    }
    // output: acc[m][n][r] = out[image img0+m][pixel po0 + r][channel 16n + i16]
    const int po0 = tile * PW_TILE + wave * 16 + kq * 4;
    uint32_t oo[NR][4];   // byte offset inside one image, BUF_OOB for masked pixels/channels
    bool valid[NR * 4];
#pragma unroll
    for (int n = 0; n < NR; n++) {
        const int ch = n * 16 + i16;
        const bool chv = ch < cout;
        const bool st = chv && stored(P, ch);
#pragma unroll
        for (int r = 0; r < 4; r++) {
            const bool pv = po0 + r < HW;
            oo[n][r] = (pv && st) ? ((uint32_t)(po0 + r) * P.out_cs + P.out_off + ch) * 4u : BUF_OOB;
            valid[n * 4 + r] = pv && chv;
        }
    }
    float rv[MI][NR][4];
    if (RES) {
        const auto rres = buf_rsrc(P.res, (uint32_t)a.B * out_img);
#pragma unroll
        for (int m = 0; m < MI; m++) {
            const uint32_t ob = img0 + m < a.B ? (uint32_t)(img0 + m) * out_img : BUF_OOB;
#pragma unroll
            for (int n = 0; n < NR; n++)
#pragma unroll
                for (int r = 0; r < 4; r++) rv[m][n][r] = buf_load1(rres, oo[n][r] == BUF_OOB ? BUF_OOB : ob + oo[n][r]);
        }
    }

    // weights -> LDS; per-image input LN (mean, rstd) -> LDS
    copy_to_lds<256>(P.wt, lw, G * 16 * NSJ);
    if (LN && wave < MI && img0 + wave < a.B) {
        float mu, rs;
        in_ln(P, img0 + wave, mu, rs);
        if (lane == 0) {
            lstat[2 * wave] = mu;
            lstat[2 * wave + 1] = rs;
        }
    }
    __syncthreads();

    f4 acc[MI][NR];
#pragma unroll
    for (int m = 0; m < MI; m++)
#pragma unroll
        for (int n = 0; n < NR; n++) acc[m][n] = f4{0.f, 0.f, 0.f, 0.f};
    float rs[MI], nmr[MI];
#pragma unroll
    for (int m = 0; m < MI; m++) {
        rs[m] = LN ? lstat[2 * m + 1] : 1.f;
        nmr[m] = LN ? -lstat[2 * m] * rs[m] : 0.f;
    }
    const float* brow = lw + ((size_t)kq * NSJ + i16) * 4;
#pragma unroll
    for (int g = 0; g < GM; g++) {
        if (g < G) {
            f4 bq[NR];
#pragma unroll
            for (int n = 0; n < NR; n++) bq[n] = *reinterpret_cast<const f4*>(brow + (size_t)g * 4 * NSJ * 4 + n * 64);
            float av[MI][4];
#pragma unroll
            for (int m = 0; m < MI; m++)
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float v = lrelu(x[m][g][j]);
                    av[m][j] = LN ? fmaf(fmaf(v, rs[m], nmr[m]), gm[g][j], bt[g][j]) : v;
                }
#pragma unroll
            for (int s = 0; s < 4; s++)
#pragma unroll
                for (int m = 0; m < MI; m++)
#pragma unroll
                    for (int n = 0; n < NR; n++)
                        acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[m][s], bq[n][s], acc[m][n], 0, 0, 0);
        }
    }
    // epilogue: bias, residual, masked store, per-wave LN partial of LeakyReLU(out)
    float bias[NR];
#pragma unroll
    for (int n = 0; n < NR; n++) bias[n] = n * 16 + i16 < cout ? P.bias[n * 16 + i16] : 0.f;
#pragma unroll
    for (int m = 0; m < MI; m++) {
        if (img0 + m >= a.B) continue;
        const int img = img0 + m;
        const uint32_t ob = (uint32_t)img * out_img;
        float vals[NR * 4];
#pragma unroll
        for (int n = 0; n < NR; n++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float v = acc[m][n][r] + bias[n];
                if (RES) v += rv[m][n][r];
                buf_store1(rout, oo[n][r] == BUF_OOB ? BUF_OOB : ob + oo[n][r], v);
                vals[n * 4 + r] = lrelu(v);
            }
        if (P.out_part != nullptr)
            ln_partial(vals, valid,
                       P.out_part + ((size_t)img * P.part_stride + P.out_part_base + tile * 4 + wave) * 3);
    }
}

void launch_pw(int nr, int gm, int mi, bool ln, bool res, const ConvArgs& a, int grid_x, int lds, hipStream_t st) {
    dim3 g(grid_x, a.nprob), b(256);
#define CNF_PW_CASE(NR_, GM_, MI_, LN_, RES_)                                                  \
    if (nr == NR_ && gm == GM_ && mi == MI_ && ln == LN_ && res == RES_) {                    \
        hipLaunchKernelGGL((k_pw<NR_, GM_, MI_, LN_, RES_>), g, b, lds, st, a);               \
        return;                                                                               \
    }
#define CNF_PW_NR(GM_, MI_, LN_, RES_)                                                        \
    CNF_PW_CASE(1, GM_, MI_, LN_, RES_) CNF_PW_CASE(2, GM_, MI_, LN_, RES_)                   \
    CNF_PW_CASE(3, GM_, MI_, LN_, RES_) CNF_PW_CASE(4, GM_, MI_, LN_, RES_)
#define CNF_PW_GM(MI_, LN_, RES_) \
    CNF_PW_NR(1, MI_, LN_, RES_) CNF_PW_NR(2, MI_, LN_, RES_) CNF_PW_NR(4, MI_, LN_, RES_) CNF_PW_NR(8, 2, LN_, RES_)
    // MI = 4 for K <= 64 without residual, else 2 (register budget of 2 waves/SIMD, pw_images())
    CNF_PW_GM(4, true, false) CNF_PW_GM(2, true, true) CNF_PW_GM(4, false, false) CNF_PW_GM(2, false, true)
#undef CNF_PW_GM
#undef CNF_PW_NR
#undef CNF_PW_CASE
    throw std::invalid_argument("k_pw: no instantiation for this shape");
}

}  // namespace cnf
