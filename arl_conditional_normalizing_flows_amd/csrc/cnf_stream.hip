// cnf_stream.hip — image-looping streamed convolutions for coupling layers whose s,t-net
// activations do not fit one CU's LDS (k_net_lds covers the rest).
//
//   k_pw   1x1 convolution (conv_a / conv_b of dilated_residual_block,
//          conv_cINN_base_functions.py:561-565, 609-613) with LeakyReLU -> per-image LayerNorm
//          (per-element gamma/beta, :330-362) applied on load, bias + residual in the epilogue
//          and the per-wave LN partials of LeakyReLU(out) for the next LayerNorm.
//
// Work decomposition: a workgroup (PW_NW waves, 16 pixels each) owns one 64-pixel tile of one net
// and loops over `ipw` images. Every wave runs its own image loop without barriers: the next
// image's activations (and residual) are loaded into registers before the current image's MFMAs,
// so HBM traffic and compute overlap inside the wave. The tile's LN gamma/beta are loaded once and
// serve every image; weights and the per-image LN (mean, rstd) live in LDS.
#include <cstdlib>
#include <cstring>
#include <stdexcept>

#include "cnf_device.h"

namespace cnf {

#include "cnf_pw_shapes.inc"   // shape-specialised k_pw instantiations (gen_netlds_shapes.py)

constexpr int PW_LDS_STAT = 256;    // byte offset of the per-image (mean, rstd) table
constexpr int PW_NW = 4;   // waves per k_pw workgroup (two workgroups per CU)

#ifndef CNF_PW_MINW
#define CNF_PW_MINW 2
#endif
// shape fields: compile-time constants of table entry SID in the shape-specialised instantiations
#define PP(f) (SID >= 0 ? kPwShapes[SID >= 0 ? SID : 0].f : P.f)
#define PA(f) (SID >= 0 ? kPwShapes[SID >= 0 ? SID : 0].f : a.f)
// diagnostic per-workgroup stamps (CNF_PW_STAMPS=SID builds only; never in timed runs): thread 0 of
// every workgroup of the instantiation SID records s_memrealtime at its start (0), before (1) and
// after (2) the prologue barrier and after each of its images (3 + i)
#if defined(CNF_PW_STAMPS) || defined(CNF_GC_WGSTAMPS)
constexpr int PW_ST_WG = 2048, PW_ST_N = 12;
#else
constexpr int PW_ST_WG = 1, PW_ST_N = 1;   // (no stamps in this build: a placeholder, never written)
#endif
__device__ long long g_pw_stamps[PW_ST_WG][PW_ST_N];
#ifdef CNF_PW_STAMPS
#define PWSTAMP(i)                                                                                       \
    do {                                                                                                 \
        if (SID == CNF_PW_STAMPS && threadIdx.x == 0 && (i) < PW_ST_N &&                                 \
            blockIdx.y * gridDim.x + blockIdx.x < PW_ST_WG)                                              \
            g_pw_stamps[blockIdx.y * gridDim.x + blockIdx.x][(i)] = (long long)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define PWSTAMP(i) do { } while (0)
#endif
int read_pw_stamps(long long* host) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_pw_stamps), sizeof(g_pw_stamps)) == hipSuccess ? 0 : -1;
}

// images of a wave in flight ahead of the one being computed: one. Deeper rings measured slower at
// cfg2 B=64 (two / four images: conv_a 19.1 -> 20.8 / 21.0 us, conv_out 11.9 -> 14.1 us; issued with
// the prologue's loads, slower still), and for the residual conv_b in round 2
//
// DUAL (generic non-tap instantiations of the training forward only): every output element is also
// stored densely ([HW][cout]) to P.out2 -- conv_a's full t1 saved for the backward in the same launch
template <int NR, int GM, bool LN, bool RES, int SID, bool TAP = false, bool DUAL = false>
__global__ __launch_bounds__(64 * PW_NW, CNF_PW_MINW) void k_pw(ConvArgs a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NW = PW_NW;
    PWSTAMP(0);
    const ConvProb P = a.p[blockIdx.y];
    const int HW = PA(H) * PA(W);
    const int tile = blockIdx.x % PA(tiles_per_img);
    const int img0 = (blockIdx.x / PA(tiles_per_img)) * a.ipw;
    const int nimg = min(a.ipw, a.B - img0);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int sub = wave;   // pixel subtile
    const int i16 = lane & 15, kq = lane >> 4;
    const int cin = PP(cin), G = (cin + 15) >> 4, cout = PP(cout);
    constexpr int NSJ = 16 * NR;
    float* lw = reinterpret_cast<float*>(smem + PP(lds_w_off));
    float* lstat = reinterpret_cast<float*>(smem + PW_LDS_STAT);
    // buffer resources: out-of-range offsets (BUF_OOB) load 0 / drop the store
    const uint32_t in_img = TAP ? (uint32_t)PA(uimg) * 4u : (uint32_t)HW * PP(in_cs) * 4u;
    const uint32_t out_img = (uint32_t)HW * PP(out_cs) * 4u;
    // one buffer resource per image (64-bit image base, 32-bit offsets inside the image): the batch
    // size never limits the addressing
    auto img_rsrc = [](const float* base, int img, uint32_t bytes) {
        return buf_rsrc(base + (size_t)img * (bytes >> 2), bytes);
    };

    // A operand: lane (i16, kq) feeds pixel pa, channels 16g + 4kq + s at k-step s of group g. Masks
    // are evaluated per element from shape fields (folded to constants in the specialised
    // instantiations, whose offsets then become lane base + immediate)
    const bool full_px = HW % (16 * NW) == 0;
    const int pa = tile * (16 * NW) + sub * 16 + i16;
    const bool pav = full_px || pa < HW;
    const uint32_t aoff = ((uint32_t)pa * PP(in_cs) + PP(in_off) + 4 * kq) * 4u;
    // mapped input (conv_b over a t2 split into its producers' sub-tensors): quad 4g + kq of the
    // lane's pixel at in_map's (offset, pixel stride)
    uint32_t amap[GM];
#pragma unroll
    for (int g = 0; g < GM; g++)
        amap[g] = PP(in_mapped) && 16 * g + 4 * kq < cin
                      ? (uint32_t)(P.in_map[2 * (4 * g + kq)] + pa * P.in_map[2 * (4 * g + kq) + 1]) * 4u
                      : 0u;
    auto aoffg = [&](int g) -> uint32_t { return PP(in_mapped) ? amap[g] : aoff + 64u * g; };
    auto gok = [&](int g) { return pav && g < G && (cin % 16 == 0 || 16 * g + 4 * kq < cin); };
    // output: acc[n][r] = out[pixel po0 + r][channel 16n + i16]
    const int po0 = tile * (16 * NW) + sub * 16 + kq * 4;
    const uint32_t obase = ((uint32_t)po0 * PP(out_cs) + PP(out_off) + i16) * 4u;
    const bool all_st = PP(st_mask_lo) == ~0u && PP(st_mask_hi) == ~0u;
    auto chv = [&](int n) { return cout % 16 == 0 || n * 16 + i16 < cout; };
    auto pv = [&](int r) { return full_px || po0 + r < HW; };
    // mapped stores (conv_a -> t1 of the streamed layers, Coupling::t1_map): the lane's channel of
    // group n goes to (offset of pixel 0, pixel stride) inside the image; offset < 0: not stored
    int cmo[NR], cms[NR];
#pragma unroll
    for (int n = 0; n < NR; n++) {
        cmo[n] = PP(st_compact) && n * 16 + i16 < 64 ? P.st_map[2 * (n * 16 + i16)] : -1;
        cms[n] = PP(st_compact) && n * 16 + i16 < 64 ? P.st_map[2 * (n * 16 + i16) + 1] : 0;
    }
    auto ooff = [&](int n, int r) -> uint32_t {   // byte offset inside one image, BUF_OOB when not stored
        const int ch = n * 16 + i16;
        if (PP(st_compact))
            return (pv(r) && chv(n) && cmo[n] >= 0) ? (uint32_t)(cmo[n] + (po0 + r) * cms[n]) * 4u : BUF_OOB;
        const bool st = all_st || ((ch < 32 ? (PP(st_mask_lo) >> ch) : (PP(st_mask_hi) >> (ch - 32))) & 1u) != 0u;
        return (pv(r) && chv(n) && st) ? obase + (uint32_t)(r * PP(out_cs) + 16 * n) * 4u : BUF_OOB;
    };
    // image activations (+ residual) in registers: the current image and the next
    f4 x[GM];
    float rv[NR][4];
    // tap mode: element k = 16g + 4kq + j of the lane's im2col row -> offset inside one image of u
    auto toff = [&](int g, int j) -> uint32_t {
        const int k = 16 * g + 4 * kq + j;
        if (!pav || k >= cin) return BUF_OOB;
        const int tap = k / PA(udc), c = k - tap * PA(udc);
        const int d = PA(udil);
        const int pr = pa / PA(W) + (tap / 3 - 1) * d, pc = pa % PA(W) + (tap % 3 - 1) * d;
        if ((unsigned)pr >= (unsigned)PA(H) || (unsigned)pc >= (unsigned)PA(W)) return BUF_OOB;
        if (PA(umask) < 0) return (uint32_t)((pr * PA(W) + pc) * PA(uD) + PA(uoff) + c) * 4u;
        return (uint32_t)mask_pos(PA(umask), pr * PA(W) + pc, c, PA(W), PA(uW), PA(uD)) * 4u;
    };
    // plain-NHWC tap sources with quad-aligned channels: one 16-byte load per (tap, quad) (the
    // row's channel quads never straddle two taps when cin % 4 == 0)
    const bool tquad = TAP && PA(umask) < 0 && PA(udc) % 4 == 0 && PA(uoff) % 4 == 0 && PA(uD) % 4 == 0;
    auto load_img = [&](int ii, f4 (&xd)[GM], float (&rd)[NR][4]) {
        const auto rin = img_rsrc(P.in, img0 + ii, in_img);
        constexpr uint32_t ib = 0;
        if constexpr (TAP) {
#pragma unroll
            for (int g = 0; g < GM; g++) {
                if (tquad) {   // the lane's 4 elements are one channel quad of one tap's pixel
                    const uint32_t o = g < G ? toff(g, 0) : BUF_OOB;
                    xd[g] = buf_load4(rin, o == BUF_OOB ? BUF_OOB : ib + o);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint32_t o = g < G ? toff(g, j) : BUF_OOB;
                        xd[g][j] = buf_load1(rin, o == BUF_OOB ? BUF_OOB : ib + o);
                    }
                }
            }
        } else {
#pragma unroll
            for (int g = 0; g < GM; g++) xd[g] = buf_load4(rin, gok(g) ? ib + aoffg(g) : BUF_OOB);
        }
        if (RES) {
            const auto rres = img_rsrc(RES ? P.res : P.out, img0 + ii, out_img);
            constexpr uint32_t ob = 0;
#pragma unroll
            for (int n = 0; n < NR; n++)
#pragma unroll
                for (int r = 0; r < 4; r++) {
                    const uint32_t o = ooff(n, r);
                    rd[n][r] = buf_load1(rres, o == BUF_OOB ? BUF_OOB : ob + o);
                }
        }
    };
    if (0 < nimg) load_img(0, x, rv);
    f4 gm[GM], bt[GM];
    if (LN) {
        const auto rg = buf_rsrc(P.gamma, in_img), rb = buf_rsrc(P.beta, in_img);
#pragma unroll
        for (int g = 0; g < GM; g++) {
            if constexpr (TAP) {   // the lane's im2col row: gamma / beta of every tap's pixel (0 outside: zero padding)
                if (tquad) {
                    const uint32_t o = g < G ? toff(g, 0) : BUF_OOB;
                    gm[g] = buf_load4(rg, o);
                    bt[g] = buf_load4(rb, o);
                } else {
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const uint32_t o = g < G ? toff(g, j) : BUF_OOB;
                        gm[g][j] = buf_load1(rg, o);
                        bt[g][j] = buf_load1(rb, o);
                    }
                }
            } else {
                const uint32_t o = gok(g) ? aoffg(g) : BUF_OOB;   // 0 where masked: the normalised value is then exactly 0
                gm[g] = buf_load4(rg, o);
                bt[g] = buf_load4(rb, o);
            }
        }
    }
    float bias[NR];
#pragma unroll
    for (int n = 0; n < NR; n++) bias[n] = n * 16 + i16 < cout ? P.bias[n * 16 + i16] : 0.f;

    // the first image of this wave's LN-statistics share: its partial slots fetched now, in the same
    // memory round trip as the loads above and the weights below (folded after the weight copy)
    const bool lnpre = LN && wave < nimg;   // (image wave: the LN table below is per workgroup)
    const LnSlots slot0 = lnpre ? in_ln_fetch(P, img0 + wave) : LnSlots{};
    // weights -> LDS; per-image input LN (mean, rstd) -> LDS
    int nwf = __builtin_amdgcn_readfirstlane(G * 16 * NSJ);
    asm volatile("" : "+s"(nwf));   // opaque count: a constant one unrolls the copy into the live image loads
    copy_to_lds<64 * NW>(P.wt, lw, nwf);
    if (LN) {
        for (int i = wave; i < nimg; i += NW) {
            float mu, rs;
            if (i == wave && lnpre)
                in_ln_finish(P, img0 + i, slot0, mu, rs);
            else
                in_ln(P, img0 + i, mu, rs);
            if (lane == 0) {
                lstat[2 * i] = mu;
                lstat[2 * i + 1] = rs;
            }
        }
    }
    PWSTAMP(1);
    __syncthreads();
    PWSTAMP(2);

    const float* brow = lw + ((size_t)kq * NSJ + i16) * 4;
    // one image: A operand from xc / rc, which then receive image pf (when it exists)
    auto step = [&](int ii, f4 (&xc)[GM], float (&rc)[NR][4], int pf) {
        const int img = img0 + ii;
        const float rs = LN ? lstat[2 * ii + 1] : 1.f;
        const float nmr = LN ? -lstat[2 * ii] * rs : 0.f;
        float av[GM][4];
#pragma unroll
        for (int g = 0; g < GM; g++) {
#pragma unroll
            for (int j = 0; j < 4; j++) {
                const float v = !TAP || P.act ? lrelu(xc[g][j]) : xc[g][j];   // conv_in reads raw u
                av[g][j] = LN ? fmaf(fmaf(v, rs, nmr), gm[g][j], bt[g][j]) : v;
            }
        }
        float res[NR][4];
        if (RES) {
#pragma unroll
            for (int n = 0; n < NR; n++)
#pragma unroll
                for (int r = 0; r < 4; r++) res[n][r] = rc[n][r];
        }
#ifndef CNF_ABL_PW_NOLOAD
        if (pf < nimg) load_img(pf, xc, rc);   // in flight during this image's MFMAs and stores
#endif
        f4 acc[NR];
#pragma unroll
        for (int n = 0; n < NR; n++) acc[n] = f4{0.f, 0.f, 0.f, 0.f};
        // B quads double-buffered one group ahead; the scheduling fence per group keeps the
        // compiler from hoisting every group's LDS reads (NR quads each) into live registers
        // (the generic instantiations keep the plain per-group loop: their runtime group bound already
        // limits the hoisting, and the extra buffer costs them registers)
        // B quads of the specialised instantiations read one group ahead (two groups ahead measured
        // no better: the LDS reads are not what each MFMA group waits on)
        constexpr int BQD = 1;
        f4 bq[BQD + 1][NR];
#pragma unroll
        for (int j = 0; j < BQD; j++)
            if (j < GM && (SID >= 0 || j == 0))
#pragma unroll
                for (int n = 0; n < NR; n++) bq[j][n] = *reinterpret_cast<const f4*>(brow + (size_t)j * 4 * NSJ * 4 + n * 64);
#pragma unroll
        for (int g = 0; g < GM; g++) {
            if (SID < 0 && g < G) {
                f4 bp[NR];
#pragma unroll
                for (int n = 0; n < NR; n++) bp[n] = *reinterpret_cast<const f4*>(brow + (size_t)g * 4 * NSJ * 4 + n * 64);
#pragma unroll
                for (int s = 0; s < 4; s++)
#pragma unroll
                    for (int n = 0; n < NR; n++)
                        acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[g][s], bp[n][s], acc[n], 0, 0, 0);
            } else if (SID >= 0 && g < G) {
                if (g + BQD < GM && g + BQD < G)
#pragma unroll
                    for (int n = 0; n < NR; n++)
                        bq[(g + BQD) % (BQD + 1)][n] =
                            *reinterpret_cast<const f4*>(brow + (size_t)(g + BQD) * 4 * NSJ * 4 + n * 64);
#pragma unroll
                for (int s = 0; s < 4; s++)
#pragma unroll
                    for (int n = 0; n < NR; n++)
                        acc[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[g][s], bq[g % (BQD + 1)][n][s], acc[n], 0, 0, 0);
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        // epilogue: bias, residual, masked store, per-wave LN partial of LeakyReLU(out)
        const auto rout = img_rsrc(P.out, img, out_img);
        const auto rout2 = img_rsrc(DUAL ? P.out2 : P.out, img, (uint32_t)HW * cout * 4u);
        constexpr uint32_t ob = 0;
        float vals[NR * 4];
        bool valid[NR * 4];
#pragma unroll
        for (int n = 0; n < NR; n++)
#pragma unroll
            for (int r = 0; r < 4; r++) {
                float v = acc[n][r] + bias[n];
                if (RES) v += res[n][r];
#ifndef CNF_ABL_PW_NOSTORE
                const uint32_t o = ooff(n, r);
                buf_store1(rout, o == BUF_OOB ? BUF_OOB : ob + o, v);
                if constexpr (DUAL)
                    buf_store1(rout2, pv(r) && chv(n) ? (uint32_t)((po0 + r) * cout + 16 * n + i16) * 4u : BUF_OOB, v);
#endif
                vals[n * 4 + r] = lrelu(v);
                valid[n * 4 + r] = pv(r) && chv(n);
            }
        if (P.out_part != nullptr)
            ln_partial(vals, valid,
                       P.out_part + ((size_t)img * PP(part_stride) + P.out_part_base + tile * NW + sub) * LNP);
    };
    // this wave's images: the buffers then receive image ii + 1
    for (int ii = 0; ii < nimg; ii++) {
        step(ii, x, rv, ii + 1);
        PWSTAMP(3 + ii);
    }
}

#undef PP
#undef PA

template <int S>
bool launch_pw_shape(int sid, const ConvArgs& a, dim3 g, dim3 b, int lds, hipStream_t st) {
    if constexpr (S < CNF_PW_NSHAPES) {
        if (sid == S) {
            constexpr PwShape k = kPwShapes[S];
            CNF_LAUNCH((k_pw<k.nr, k.gm, k.ln != 0, k.res != 0, S, k.tap != 0>), g, b, lds, st, a);
            return true;
        }
        return launch_pw_shape<S + 1>(sid, a, g, b, lds, st);
    }
    return false;
}

int pw_num_shapes() { return CNF_PW_NSHAPES; }

void launch_pw(int nr, int gm, bool ln, bool res, bool tap, const ConvArgs& a, int grid_x, int lds, hipStream_t st) {
    dim3 g(grid_x, a.nprob), b(64 * PW_NW);
    const bool generic = opts().generic != 0;   // debug option GENERIC=1
    bool dual = false;
    for (int i = 0; i < a.nprob; i++) dual |= a.p[i].out2 != nullptr;
    if (dual) {   // training forward conv_a with the dense t1 copy: generic instantiations only
        if (tap || res || !ln) throw std::invalid_argument("k_pw dual store: LN, no residual, no tap mode");
        for (int i = 0; i < a.nprob; i++)
            if (a.p[i].out2 == nullptr) throw std::invalid_argument("k_pw dual store: every problem needs out2");
#define CNF_PW_DCASE(NR_, GM_)                                                         \
        if (nr == NR_ && gm == GM_) {                                                  \
            CNF_LAUNCH((k_pw<NR_, GM_, true, false, -1, false, true>), g, b, lds, st, a); \
            return;                                                                    \
        }
#define CNF_PW_DNR(GM_) CNF_PW_DCASE(1, GM_) CNF_PW_DCASE(2, GM_) CNF_PW_DCASE(3, GM_) CNF_PW_DCASE(4, GM_)
        CNF_PW_DNR(1) CNF_PW_DNR(2) CNF_PW_DNR(4) CNF_PW_DNR(8)
#undef CNF_PW_DNR
#undef CNF_PW_DCASE
        throw std::invalid_argument("k_pw dual store: no instantiation for this shape");
    }
    PwShape sh;
    if (!generic && pw_shape_of(nr, gm, ln, res, tap, a, sh))
        for (int sid = 0; sid < CNF_PW_NSHAPES; sid++)
            if (std::memcmp(&sh, &kPwShapes[sid], sizeof(sh)) == 0 && launch_pw_shape<0>(sid, a, g, b, lds, st)) return;
    if (tap) {   // generic tap mode (streamed conv_in / grouped branches): no residual, K <= 128
        if (res || gm > 8) throw std::invalid_argument("k_pw tap mode: no residual, K <= 128");
#define CNF_PW_TCASE(NR_, GM_, LN_)                                                     \
        if (nr == NR_ && gm == GM_ && ln == LN_) {                                      \
            CNF_LAUNCH((k_pw<NR_, GM_, LN_, false, -1, true>), g, b, lds, st, a); \
            return;                                                                     \
        }
#define CNF_PW_TNR(GM_, LN_) CNF_PW_TCASE(1, GM_, LN_) CNF_PW_TCASE(2, GM_, LN_) CNF_PW_TCASE(3, GM_, LN_) CNF_PW_TCASE(4, GM_, LN_)
        CNF_PW_TNR(1, false) CNF_PW_TNR(2, false) CNF_PW_TNR(4, false) CNF_PW_TNR(8, false)
        CNF_PW_TNR(1, true) CNF_PW_TNR(2, true) CNF_PW_TNR(4, true) CNF_PW_TNR(8, true)
#undef CNF_PW_TNR
#undef CNF_PW_TCASE
        throw std::invalid_argument("k_pw tap mode: no instantiation for this shape");
    }
#define CNF_PW_CASE(NR_, GM_, LN_, RES_)                                              \
    if (nr == NR_ && gm == GM_ && ln == LN_ && res == RES_) {                          \
        CNF_LAUNCH((k_pw<NR_, GM_, LN_, RES_, -1>), g, b, lds, st, a);             \
        return;                                                                        \
    }
#define CNF_PW_NR(GM_, LN_, RES_) \
    CNF_PW_CASE(1, GM_, LN_, RES_) CNF_PW_CASE(2, GM_, LN_, RES_) CNF_PW_CASE(3, GM_, LN_, RES_) CNF_PW_CASE(4, GM_, LN_, RES_)
#define CNF_PW_GM(LN_, RES_) CNF_PW_NR(1, LN_, RES_) CNF_PW_NR(2, LN_, RES_) CNF_PW_NR(4, LN_, RES_) CNF_PW_NR(8, LN_, RES_)
    CNF_PW_GM(true, false) CNF_PW_GM(false, false) CNF_PW_GM(true, true) CNF_PW_GM(false, true)
#undef CNF_PW_GM
#undef CNF_PW_NR
#undef CNF_PW_CASE
    throw std::invalid_argument("k_pw: no instantiation for this shape");
}

}  // namespace cnf

namespace cnf {

#include "cnf_gc_shapes.inc"   // shape-specialised k_gc instantiations (gen_netlds_shapes.py)

// ---------------------------------------------------------------------------------------------
// k_gc: the grouped dilated stage of a residual block (conv_cINN_base_functions.py:364-413,
// 583-601) for the streamed layers — LN2(LeakyReLU(t1)) on the branch windows -> every branch's
// dense 3x3 dilated conv -> t2 slices, plus the per-wave LN3 partials of LeakyReLU(t2).
// ---------------------------------------------------------------------------------------------
// waves / threads of the instantiation for table entry SID (-1: generic)
#define GC_NWS (SID >= 0 ? kGcShapes[SID >= 0 ? SID : 0].nw : GC_NW_GEN)
#define GC_NTS (64 * GC_NWS)

// shape fields: compile-time constants of table entry SID in the shape-specialised instantiations
#define GS(f) (SID >= 0 ? kGcShapes[SID >= 0 ? SID : 0].f : a.s.f)

// BI >= 0 (specialised instantiations): branch BI of table entry SID, every field a constant
// tile pixel -> image pixel: full-width / 2-D tiles (ps == 1: px0 + row * W + column), or polyphase
// tiles (block blk of the tile = phase grid ph0 + blk, pixel (r0 + row, column) of that grid)
template <int SID>
__device__ __forceinline__ int gc_out_pixel(const GcArgs& a, int po, int px0, int r0, int ph0) {
    const int tpx = GS(TH) * GS(TW);
    const int blk = GS(nbk) > 1 ? po / tpx : 0;
    const int rem = po - blk * tpx;
    const int por = rem / GS(TW), poc = rem - por * GS(TW);
    if (GS(ps) > 1) {
        const int ph = ph0 + blk, pa = ph / GS(ps), pb = ph - pa * GS(ps);
        return (pa + (r0 + por) * GS(ps)) * GS(W) + pb + poc * GS(ps);
    }
    return px0 + por * GS(W) + poc;
}

template <int NR, int SID, int BI>
__device__ __forceinline__ void gc_branch(const GcArgs& a, const GcBranch& brx, const unsigned char* smem,
                                          const float* bias, float* __restrict__ outp, int npx,
                                          int px0, int r0, int ph0, LnAcc& st, bool& first, bool stats, int boff) {
    const GcBranch& br = BI >= 0 ? kGcShapes[SID >= 0 ? SID : 0].br[BI >= 0 ? BI : 0] : brx;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int i16 = lane & 15, kq = lane >> 4;
    constexpr int NSJ = 16 * NR;
    const float* band = reinterpret_cast<const float*>(smem + br.band_off + boff);
    const float* lw = reinterpret_cast<const float*>(smem + br.w_off);
    const int* qo = reinterpret_cast<const int*>(smem + br.q_off);
    // operands swapped (A = weights, B = activations): lane (i16, kq) ends with pixel i16, channels
    // 16n + 4kq + r (r < 4) of the subtile, i.e. one 16-byte channel quad per n -> f4 stores
    f4 bz[NR];
    int nq[NR];   // valid channels of the lane's quad (0..4)
#pragma unroll
    for (int n = 0; n < NR; n++) {
        const int c0 = n * 16 + 4 * kq;
        nq[n] = max(0, min(4, br.cout - c0));
#pragma unroll
        for (int r = 0; r < 4; r++) bz[n][r] = r < nq[n] ? bias[c0 + r] : 0.f;
    }
    const bool vq = ((br.opcs | br.out_off) & 3) == 0;
    const int nsub = (npx + 15) >> 4;
    // two subtiles per wave and pass (s0, s0 + NW) share every B read: two independent MFMA
    // chains per wave keep the SIMD busy at 2 waves per SIMD; A quads are issued in chunks of GQ
    constexpr int GQ = 6;
    const int G = br.G;
    const float* brow = lw + ((size_t)kq * NSJ + i16) * 4;
    constexpr int NW = GC_NWS;   // (16 waves cover a 256-pixel tile in one pass: the pair's second half is dead code)
    for (int s0 = wave; s0 < nsub; s0 += 2 * NW) {
        const int s1 = s0 + NW;
        const bool v1 = s1 < nsub;
        const float* base[2];
#pragma unroll
        for (int h = 0; h < 2; h++) {
            const int pt = (h ? s1 : s0) * 16 + i16;
            const int ptc = pt < npx ? pt : 0;
            // block blk of a polyphase tile: band rows [blk (TH + 2 dil), ...)
            const int tpx = GS(TH) * GS(TW);
            const int blk = GS(nbk) > 1 ? ptc / tpx : 0;
            const int rem = ptc - blk * tpx;
            const int tr = rem / GS(TW), tc = rem - tr * GS(TW);
            base[h] = band + ((blk * (GS(TH) + 2 * br.dil) + tr) * br.BW + tc) * br.S;
        }
        f4 acc0[NR], acc1[NR];   // start at the bias
#pragma unroll
        for (int n = 0; n < NR; n++) {
            acc0[n] = bz[n];
            acc1[n] = bz[n];
        }
        for (int g0 = 0; g0 < G; g0 += GQ) {
            int qv[GQ];
#pragma unroll
            for (int j = 0; j < GQ; j++) qv[j] = g0 + j < G ? qo[4 * (g0 + j) + kq] : 0;
            f4 a0[GQ], a1[GQ];
#pragma unroll
            for (int j = 0; j < GQ; j++) {
                a0[j] = *reinterpret_cast<const f4*>(base[0] + qv[j]);
                a1[j] = *reinterpret_cast<const f4*>(base[1] + qv[j]);
            }
#pragma unroll
            for (int j = 0; j < GQ; j++) {
                if (g0 + j >= G) break;
                const int g = g0 + j;
                f4 bq[NR];
#pragma unroll
                for (int n = 0; n < NR; n++) bq[n] = *reinterpret_cast<const f4*>(brow + (size_t)g * 4 * NSJ * 4 + n * 64);
#pragma unroll
                for (int q = 0; q < 4; q++)
#pragma unroll
                    for (int n = 0; n < NR; n++) {
                        acc0[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(bq[n][q], a0[j][q], acc0[n], 0, 0, 0);
                        acc1[n] = __builtin_amdgcn_mfma_f32_16x16x4f32(bq[n][q], a1[j][q], acc1[n], 0, 0, 0);
                    }
            }
        }
        if (stats && first) {
            st.set_shift(lrelu(acc0[0][0]));
            first = false;
        }
#pragma unroll
        for (int h = 0; h < 2; h++) {
            if (h == 1 && !v1) break;
            const int po = (h ? s1 : s0) * 16 + i16;
            const bool pv = po < npx;
            float* orow = outp + (size_t)gc_out_pixel<SID>(a, pv ? po : 0, px0, r0, ph0) * br.opcs + br.out_off + 4 * kq;
#pragma unroll
            for (int n = 0; n < NR; n++) {
                const f4 v = h ? acc1[n] : acc0[n];
#ifdef CNF_ABL_GC_NOSTORE_POLY   // ablation (diagnostic builds only): no t2 stores from polyphase tiles
                if (GS(ps) > 1) {
                } else
#endif
                if (pv && nq[n] == 4 && vq) {
                    *reinterpret_cast<f4*>(orow + n * 16) = v;
                } else if (pv) {
#pragma unroll
                    for (int r = 0; r < 4; r++)
                        if (r < nq[n]) orow[n * 16 + r] = v[r];
                }
                if (stats) {
#pragma unroll
                    for (int r = 0; r < 4; r++) st.add(lrelu(v[r]), pv && r < nq[n]);
                }
            }
        }
    }
}

// staged band quads per thread: 2 in the specialised instantiations (the plan keeps a group's bands
// within 128 quads per wave), GC_STAGE_QUADS over the generic kernel's threads
#define GC_GQS (SID >= 0 ? 2 : GC_STAGE_QUADS / GC_NTS)
#define GC_PDS (SID >= 0 ? kGcShapes[SID >= 0 ? SID : 0].pd : 1)   // band prefetch depth (images)

// the branches of table entry SID, unrolled at compile time
template <int SID, int BI>
__device__ __forceinline__ void gc_branches(const GcArgs& a, const unsigned char* smem, float* __restrict__ outp,
                                            int npx, int px0, int r0, int ph0, LnAcc& st, bool& first, bool stats,
                                            int boff) {
    if constexpr (BI < kGcShapes[SID].nbr) {
        constexpr GcBranch br = kGcShapes[SID].br[BI];
        const float* bias = reinterpret_cast<const float*>(smem + br.b_off);
        gc_branch<(br.cout + 15) / 16, SID, BI>(a, br, smem, bias, outp, npx, px0, r0, ph0, st, first, stats, boff);
        gc_branches<SID, BI + 1>(a, smem, outp, npx, px0, r0, ph0, st, first, stats, boff);
    }
}

// diagnostic phase stamps of workgroup (0, 0) (CNF_GC_STAMPS builds only; never in timed runs)
__device__ long long g_gc_stamps[64];
#ifdef CNF_GC_STAMPS
#define GSTAMP(i)                                                                             \
    do {                                                                                      \
        __syncthreads();                                                                      \
        if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0)                           \
            g_gc_stamps[(i)] = (long long)__builtin_amdgcn_s_memrealtime();                  \
    } while (0)
#else
#define GSTAMP(i) do { } while (0)
#endif
// per-workgroup stamps (CNF_GC_WGSTAMPS builds only): thread 0 of every workgroup, at its start (0),
// after the prologue (1) and after each image (2 + i); read through cnf_debug_read_pw_stamps
#ifdef CNF_GC_WGSTAMPS
#define GWSTAMP(i)                                                                                       \
    do {                                                                                                 \
        if (threadIdx.x == 0 && (i) < PW_ST_N && blockIdx.y * gridDim.x + blockIdx.x < PW_ST_WG)         \
            g_pw_stamps[blockIdx.y * gridDim.x + blockIdx.x][(i)] = (long long)__builtin_amdgcn_s_memrealtime(); \
    } while (0)
#else
#define GWSTAMP(i) do { } while (0)
#endif

// One workgroup per CU: a tile of TH rows of one net, looping over `ipw` images. The bands are
// double-buffered: the next image's t1 quads are loaded into registers before the current image's
// MFMAs and written (LN2 + LeakyReLU applied) into the other buffer after them, so the staging
// latency hides behind the compute; the tile's LN2 gamma/beta stay in registers for all images.
template <int SID>
__global__ __launch_bounds__(GC_NTS, SID >= 0 ? 16 / GC_NWS : 1) void k_gc(GcArgs a) {
    constexpr int GC_NW = GC_NWS, GC_NT = GC_NTS, GC_GQ = GC_GQS, PD = GC_PDS;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int net = blockIdx.y;
    const int tile = blockIdx.x % GS(tiles_per_img);
    const int img0 = (blockIdx.x / GS(tiles_per_img)) * a.ipw;
    const int nimg = min(a.ipw, a.B - img0);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int H = GS(H), W = GS(W), HW = H * W;
    // 2-D tiles: TH rows x TW columns (TW == W for all but the widest images; W % TW == 0); polyphase
    // tiles (ps > 1): nbk phase grids from ph0, rows [r0, r0 + TH) of each (tpp row slices per grid)
    const bool poly = GS(ps) > 1;
    const int ty = GS(tiles_x) == 1 ? tile : tile / GS(tiles_x), tx = tile - ty * GS(tiles_x);
    const int ph0 = poly ? (tile / GS(tpp)) * GS(nbk) : 0;
    const int r0 = poly ? (tile - (tile / GS(tpp)) * GS(tpp)) * GS(TH) : ty * GS(TH), c0 = poly ? 0 : tx * GS(TW);
    const int rows = poly || GS(H) % GS(TH) == 0 ? GS(TH) : min(GS(TH), H - r0);
    const int npx = GS(nbk) * rows * GS(TW), px0 = r0 * W + c0;
    const bool ln = SID >= 0 ? (GS(lnst) & 1) != 0 : a.in_part[net] != nullptr;
    const bool stats = SID >= 0 ? (GS(lnst) & 2) != 0 : a.out_part[net] != nullptr;
    float* lstat = reinterpret_cast<float*>(smem + PW_LDS_STAT);
    float* lds_f = reinterpret_cast<float*>(smem);
    int gs = 0;
    GSTAMP(gs++);
    GWSTAMP(0);

    // image-independent staging plan of this thread: quad e = tid + GC_NT*u of the concatenated branch
    // bands -> source offset inside one image, LDS float index, valid channels (0 = zero quad)
    int soff[GC_GQ], loff[GC_GQ], nv[GC_GQ];
#pragma unroll
    for (int u = 0; u < GC_GQ; u++) {
        int e = tid + GC_NT * u;
        soff[u] = 0;
        loff[u] = -1;
        nv[u] = 0;
        for (int bi = 0; bi < GS(nbr); bi++) {
            const GcBranch& br = GS(br)[bi];
            const int cpq = br.cinp >> 2, nq = br.BH * br.BW * cpq;
            if (e < nq) {
                const int pix = cpq == 1 ? e : (int)__umulhi((unsigned)e, br.cpq_mag), cq = e - pix * cpq;
                const int brr = (int)__umulhi((unsigned)pix, br.bw_mag), bc = pix - brr * br.BW;
                int y = r0 - br.dil + brr, x = c0 + bc - br.dil;
                bool inb = y >= 0 && y < H && x >= 0 && x < W;
                if (poly) {   // band row brr of block blk -> row of phase grid ph0 + blk
                    const int bh = GS(TH) + 2, blk = brr / bh, sy = r0 - 1 + brr - blk * bh, sx = bc - 1;
                    const int ph = ph0 + blk, pa = ph / GS(ps), pb = ph - pa * GS(ps);
                    inb = sy >= 0 && sy < H / GS(ps) && sx >= 0 && sx < W / GS(ps);
                    y = pa + sy * GS(ps);
                    x = pb + sx * GS(ps);
                }
                loff[u] = br.band_off / 4 + pix * br.S + 4 * cq;
                if (inb) {
                    soff[u] = (y * W + x) * br.pcs + br.cin_off + 4 * cq;
                    const int v = min(4, br.cin - 4 * cq);
                    const bool vec = v == 4 && ((br.cin_off | br.pcs) & 3) == 0;
                    nv[u] = v | (vec ? 8 : 0);
                }
                break;
            }
            e -= nq;
        }
    }
    // one staged quad through a buffer resource (out-of-range offset BUF_OOB reads 0). The vector
    // / scalar choice is made per wave (ballot), never per lane: a lane-divergent choice makes both
    // paths write the same VGPRs, and the compiler then drains every load (vmcnt(0)) before the next
    // one — the gathers of a band would run one round trip at a time.
    auto load_q = [&](__amdgpu_buffer_rsrc_t r, int u) -> f4 {
        const int n = nv[u] & 7;
        const uint32_t o = (uint32_t)soff[u] * 4u;
        if (__all(n == 0 || (nv[u] & 8) != 0)) return buf_load4(r, n == 0 ? BUF_OOB : o);
        f4 v;
#pragma unroll
        for (int j = 0; j < 4; j++) v[j] = buf_load1(r, j < n ? o + 4u * j : BUF_OOB);
        return v;
    };
    const uint32_t img_bytes = (uint32_t)HW * GS(in_cs) * 4u;
    // tile LN2 gamma/beta (image-independent) and the first image's raw quads, all in flight together
    f4 gq[GC_GQ], bq[GC_GQ], xq[PD][GC_GQ];   // xq: a ring of PD images' raw quads
#pragma unroll
    for (int u = 0; u < GC_GQ; u++) {
        gq[u] = ln ? load_q(buf_rsrc(a.gamma[net], img_bytes), u) : f4{1.f, 1.f, 1.f, 1.f};
        bq[u] = ln ? load_q(buf_rsrc(a.beta[net], img_bytes), u) : f4{0.f, 0.f, 0.f, 0.f};
    }
    auto load_img = [&](int ii, f4 (&xd)[GC_GQ]) {
        const auto r = buf_rsrc(a.in[net] + (size_t)(img0 + ii) * HW * GS(in_cs), img_bytes);
#pragma unroll
        for (int u = 0; u < GC_GQ; u++) xd[u] = load_q(r, u);
    };
    // LN2(LeakyReLU(t1)) of the quads in xq -> band buffer (ii & 1); zero outside the image / window
    auto store_img = [&](int ii, const f4 (&xs)[GC_GQ]) {
        const float rs = ln ? lstat[2 * ii + 1] : 1.f;
        const float nmr = ln ? -lstat[2 * ii] * rs : 0.f;
        float* dst = lds_f + (ii & 1) * (GS(band_bytes) / 4);
#pragma unroll
        for (int u = 0; u < GC_GQ; u++) {
            if (loff[u] < 0) continue;
            f4 v = f4{0.f, 0.f, 0.f, 0.f};
            if (nv[u] != 0) {
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const float t = lrelu(xs[u][j]);
                    v[j] = ln ? fmaf(fmaf(t, rs, nmr), gq[u][j], bq[u][j]) : t;
                }
            }
            *reinterpret_cast<f4*>(dst + loff[u]) = v;
        }
    };
    load_img(0, xq[0]);
    // this wave's first LN2 image: partial slots fetched in the same memory round trip as the band
    // and weight loads (folded below)
    ConvProb lnP;
    lnP.in_part = a.in_part[net];
    lnP.in_nparts = a.in_nparts;
    lnP.part_stride = a.part_stride;
    const bool lnpre = ln && wave < nimg;
    const LnSlots slot0 = lnpre ? in_ln_fetch(lnP, img0 + wave) : LnSlots{};
    // packed weights and quad-offset tables of every branch (once per workgroup)
    for (int bi = 0; bi < GS(nbr); bi++) {
        const GcBranch& br = GS(br)[bi];
        const int nr = (br.cout + 15) >> 4;
        copy_to_lds<GC_NT>(a.w[net][bi], reinterpret_cast<float*>(smem + br.w_off), br.G * 16 * 16 * nr);
        for (int i = tid; i < br.cout; i += GC_NT) reinterpret_cast<float*>(smem + br.b_off)[i] = a.b[net][bi][i];
        int* qo = reinterpret_cast<int*>(smem + br.q_off);
        const int cpq = br.cinp >> 2, nq = 9 * cpq;
        for (int qd = tid; qd < 4 * br.G; qd += GC_NT) {
            int o = 0;   // padding quads have zero weights: any in-band address is fine
            if (qd < nq) {
                const int tap = qd / cpq, cq = qd - tap * cpq;
                o = (((tap / 3) * br.dil) * br.BW + (tap % 3) * br.dil) * br.S + 4 * cq;
            }
            qo[qd] = o;
        }
    }
    GSTAMP(gs++);   // (diagnostic builds: band / gamma / beta / weight loads landed)
    // per-image LN2 (mean, rstd) from the producer's partials
    if (ln) {
        for (int i = wave; i < nimg; i += GC_NW) {
            float mu, rs;
            if (i == wave && lnpre)
                in_ln_finish(lnP, img0 + i, slot0, mu, rs);
            else
                in_ln(lnP, img0 + i, mu, rs);
            if (lane == 0) {
                lstat[2 * i] = mu;
                lstat[2 * i + 1] = rs;
            }
        }
    }
    __syncthreads();
    store_img(0, xq[0]);
    __syncthreads();
    GSTAMP(gs++);
    GWSTAMP(1);

    // the ring's other images (PD > 1)
#pragma unroll
    for (int j = 1; j < PD; j++)
        if (j < nimg) load_img(j, xq[j]);
    for (int i0 = 0; i0 < nimg; i0 += PD)
#pragma unroll
    for (int jj = 0; jj < PD; jj++) {
        const int ii = i0 + jj;
        if (ii >= nimg) break;
        const int img = img0 + ii;
        // lands while this image's MFMAs run: the next image (PD == 1), or image ii + PD into the
        // ring slot image ii (already staged) leaves
        if (PD == 1 && ii + 1 < nimg) load_img(ii + 1, xq[0]);
        if (PD > 1 && ii + PD < nimg) load_img(ii + PD, xq[jj]);
        LnAcc st;
        st.reset();
        bool first = true;
        float* outp = a.out[net] + (size_t)img * HW * GS(out_cs);
        const int boff = (ii & 1) * GS(band_bytes);
        if constexpr (SID >= 0) {
            gc_branches<SID, 0>(a, smem, outp, npx, px0, r0, ph0, st, first, stats, boff);
        } else {
            for (int bi = 0; bi < GS(nbr); bi++) {
                const GcBranch& br = GS(br)[bi];
                const float* bias = reinterpret_cast<const float*>(smem + br.b_off);
                switch ((br.cout + 15) >> 4) {
                    case 1: gc_branch<1, SID, -1>(a, br, smem, bias, outp, npx, px0, r0, ph0, st, first, stats, boff); break;
                    case 2: gc_branch<2, SID, -1>(a, br, smem, bias, outp, npx, px0, r0, ph0, st, first, stats, boff); break;
                    case 3: gc_branch<3, SID, -1>(a, br, smem, bias, outp, npx, px0, r0, ph0, st, first, stats, boff); break;
                    default: gc_branch<4, SID, -1>(a, br, smem, bias, outp, npx, px0, r0, ph0, st, first, stats, boff); break;
                }
                GSTAMP(gs++);
            }
        }
        if (stats) st.write(a.out_part[net] + ((size_t)img * a.part_stride + tile * GC_NW + wave) * LNP);
        if (ii + 1 < nimg) store_img(ii + 1, xq[(jj + 1) % PD]);   // the other buffer: nobody reads it this iteration
        __syncthreads();
        GSTAMP(gs++);
        GWSTAMP(2 + ii);
    }
#ifdef CNF_GC_STAMPS
    if (threadIdx.x == 0 && blockIdx.x == 0 && blockIdx.y == 0) g_gc_stamps[63] = gs;
#endif
}

int read_gc_stamps(long long* host, int n) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_gc_stamps), sizeof(long long) * (n > 64 ? 64 : n)) == hipSuccess ? 0 : -1;
}

template <int S>
bool launch_gc_shape(int sid, const GcArgs& a, dim3 grid, int lds, hipStream_t st) {
    if constexpr (S < CNF_GC_NSHAPES) {
        if (sid == S) {
            CNF_LAUNCH((k_gc<S>), grid, dim3(64 * kGcShapes[S].nw), lds, st, a);
            return true;
        }
        return launch_gc_shape<S + 1>(sid, a, grid, lds, st);
    }
    return false;
}

int gc_num_shapes() { return CNF_GC_NSHAPES; }

// table entry matching a's shape, -1 for the generic instantiation
static int gc_shape_id(const GcArgs& a) {
    const bool generic = opts().generic != 0;   // debug option GENERIC=1
    if (!generic)
        for (int sid = 0; sid < CNF_GC_NSHAPES; sid++)
            if (std::memcmp(&a.s, &kGcShapes[sid], sizeof(GcShape)) == 0) return sid;
    return -1;
}

int gc_waves(const GcArgs& a) {
    const int sid = gc_shape_id(a);
    return sid >= 0 ? kGcShapes[sid].nw : GC_NW_GEN;
}

void launch_gc(const GcArgs& a, int grid_x, int lds, hipStream_t st) {
    const dim3 grid(grid_x, 2);
    const int sid = gc_shape_id(a);
    if (sid >= 0 && launch_gc_shape<0>(sid, a, grid, lds, st)) return;
    CNF_LAUNCH((k_gc<-1>), grid, dim3(64 * GC_NW_GEN), lds, st, a);
}

}  // namespace cnf
