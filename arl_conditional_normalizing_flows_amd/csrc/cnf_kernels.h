// cnf_kernels.h — kernel argument blocks and launch helpers (host <-> device contract).
#pragma once

#include <cstddef>

#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstdint>
#include <cstdlib>

namespace cnf {

constexpr float LRELU_ALPHA = 0.3f;      // keras.layers.LeakyReLU() default
constexpr float LN_EPS = 1e-3f;          // keras.layers.LayerNormalization() default
constexpr double LOG_2PI_D = 1.8378770664093453;
// LayerNorm statistics partial of one producing wave: (K, S1, S2, n) with S1 = sum(x - K),
// S2 = sum((x - K)^2) over its n values of LeakyReLU(out), K a sample of them (fp32, 16 bytes)
constexpr int LNP = 4;
// LN partial slots per image a consumer wave folds from its prologue loads, per lane (cnf_device.h
// in_ln_fetch); producers of more than 64 * LN_FETCH slots get a k_ln_merge launch (cnf_runtime.cpp)
constexpr int LN_FETCH = 8;

constexpr int MAXPROB = 12;

// Debug options of a plan: cnf_flow_desc.debug_options, "NAME=V[,NAME=V...]" (include/cnf.h). They
// select the alternative code paths the parity tests compare against the default ones; the library
// reads no environment variable, and the defaults are what bench.py measures.
struct Options {
    int netlds = 1;          // NETLDS: 0 = no LDS-resident (k_net_lds) layers, every layer streamed
    int gc = 1;              // GC: 0 = no fused k_gc stage (grouped branches as k_pw tap mode / k_conv<3>)
    int pw = 1;              // PW: 0 = the per-tile k_conv1 / k_conv<3> kernels and the one-kernel k_convtap conv_out
#ifndef CNF_DIAG_GENERIC
#define CNF_DIAG_GENERIC 0   // (diagnostic builds: a different default for A/B runs of the unmodified tests)
#endif
    int generic = CNF_DIAG_GENERIC;   // GENERIC bits: never the shape-specialised instantiations of 1 any kernel, 2 k_pw, 4 k_gc, 8 k_net_lds
    int layout = 7;          // LAYOUT bits: 1 compact t1 sub-tensors, 2 mapped t2 sub-tensors, 4 polyphase k_gc tiles
    int fuse_coupling = 1;   // FUSE_COUPLING: 0 = every coupling layer launches its own k_coupling
    int lds_bwd = 2;         // LDS_BWD: 0 multi-kernel backward of the k_net_lds layers, 1 fused (one launch), 2 fused split
    // TRAIN_ALT bits, alternative training kernels: 1 VALU convolutions, 2 LDS-staged band weight gradients
    // (no k_wgrad_direct), 4 no band-staged transposed conv, 8 no thin-channel kernels, 16 a separate
    // LN-backward reduction kernel, 32 a zeroed dt1 gradient instead of the LN2 channel mask
    int train_alt = 0;
    // TRAIN_SCHED bits: 1 weight gradients on the chain streams, 2 recompute the streamed activations
    // (no saves), 4 enqueue net A's chain before net b's (no interleaving)
    int train_sched = 0;
};
// parses a debug_options string (null / empty: defaults); throws std::invalid_argument on an unknown
// name or a malformed value (cnf_runtime.cpp)
Options parse_options(const char* s);
// the options of the plan the calling thread's current C-ABI call runs (defaults outside one)
const Options& opts();
struct OptScope {   // sets opts() for the duration of one C-ABI call
    const Options* prev;
    explicit OptScope(const Options* o);
    ~OptScope();
};

// Launch timing (bench.py via cnf_plan_set_launch_timing): while a pair is armed, the launch
// helpers dispatch through hipExtLaunchKernelGGL, which stores the kernel's own begin / end
// timestamps (the dispatch packet's profiling timestamps, as rocprofv3 reads them) into the
// events: no extra packets between the kernels, so the stream runs as it does untimed.
struct LaunchTiming {
    hipEvent_t start = nullptr, stop = nullptr;
    int used = 0;   // kernels that wrote the pair (the last one's times are kept)
};
LaunchTiming& launch_timing();   // per host thread (cnf_runtime.cpp)
#define CNF_LAUNCH(K, G, B, L, S, ...)                                                              \
    do {                                                                                            \
        ::cnf::LaunchTiming& lt_ = ::cnf::launch_timing();                                          \
        if (lt_.start != nullptr) {                                                                 \
            hipExtLaunchKernelGGL(K, G, B, L, S, lt_.start, lt_.stop, 0, __VA_ARGS__);              \
            lt_.used++;                                                                             \
        } else {                                                                                    \
            hipLaunchKernelGGL(K, G, B, L, S, __VA_ARGS__);                                         \
        }                                                                                           \
        CNF_DIAG_SYNC(S);                                                                           \
    } while (0)
#ifdef CNF_DIAG   // diagnostic builds: CNF_SYNC_ALL=1 synchronises the stream after every launch
#define CNF_DIAG_SYNC(S)                                                                            \
    do {                                                                                            \
        static const bool sync_ = std::getenv("CNF_SYNC_ALL") != nullptr;                          \
        if (sync_) (void)hipStreamSynchronize(S);                                                   \
    } while (0)
#else
#define CNF_DIAG_SYNC(S) do { } while (0)
#endif

// packed weight-image formats (see cnf_plan.h PackedConv)
enum { PK_1X1 = 0, PK_KN = 1, PK_TAP = 2, PK_Q4 = 3 };

// kernel roles: distinct symbols so per-kernel profiles separate the ResNeXt stages
enum { ROLE_CONV_IN = 0, ROLE_CONV_A = 1, ROLE_GC = 2, ROLE_CONV_B = 3, ROLE_CONV_OUT = 4 };

// One convolution problem of a k_conv launch (blockIdx.y selects the problem).
struct ConvProb {
    const float* in;          // NHWC, image 0
    const float* in_part;     // LN partials (K, S1, S2, n) of the input tensor [B][part_stride][LNP] (first
                              // in_nparts slots valid), or null (no LN)
    const float* gamma;       // LN gamma over the full in_cs-channel tensor (per h,w,c)
    const float* beta;
    const float* wt;          // pre-packed weight image (PK_1X1 / PK_KN / PK_TAP)
    const float* bias;        // [cout]
    const float* res;         // residual, same layout as out, or null
    float* out;
    float* out_part;          // per-wave LN partials of LeakyReLU(out) [B][part_stride][LNP], or null
    int in_cs, in_off, cin, in_nparts;
    int out_cs, out_off, cout, part_stride, out_part_base;
    int dil, act;
    int lds_in_off, lds_w_off, lds_k_off;  // byte offsets in dynamic LDS
    int S, Kpad, NS, nr;                   // LDS pixel stride, padded K, B row stride, N-subtiles
    uint32_t cin_mag, wp_mag;              // magic multipliers: x / cin == umulhi(x, cin_mag) (3x3 staging)
    uint32_t st_mask_lo, st_mask_hi;       // output channels actually stored (bit per channel < 64)
    int st_compact;                        // 1: stores through st_map (k_pw only)
    const int* st_map;                     // [64][2]: channel -> (offset of pixel 0 inside the image, pixel stride) in floats, offset < 0: not stored
    int in_mapped;                         // 1: A-operand quads through in_map (k_pw only; in_cs = floats per pixel of an image)
    const int* in_map;                     // [quad][2]: input channel quad -> (offset of pixel 0 inside the image, pixel stride)
    float* out2;                           // k_pw only: also every output channel, plain [B][HW][cout] (null: none) —
                                           // the training forward's full t1 next to conv_a's mapped stores
};

struct ConvArgs {
    ConvProb p[MAXPROB];
    int H, W, TH, tiles_per_img, nprob, B;
    int P;     // 1x1 kernels: pixels per tile (tiles are runs of pixels inside one image)
    int ipw;   // k_pw: images per workgroup (looped, next image prefetched)
    // k_pw tap mode (streamed conv_in): the A operand is the im2col row of a 3x3 conv over the
    // mask-compressed half of the raw layer input u, gathered straight from u (no u1c tensor):
    // K index k = tap * udc + c, c < udc, pixel shifted by the tap, zero outside the image
    int umask, uW, uD, udc, uimg;   // mask, full-res width / depth, channels per tap, floats per image
    // umask < 0: the source is a plain NHWC tensor of the conv's own H x W (uD channels per pixel,
    // taps from channel uoff, dilation udil; LN / LeakyReLU on load as the problem says)
    int udil, uoff;
    int diag;   // -DCNF_DIAG builds only: k_pw experiment bits (CNF_PW_DIAG)
};

struct CoupArgs {
    const float* u;
    float* v;
    const float* s_pre;      // raw conv_out of net A (before tanh)
    const float* t;          // conv_out of net b
    const float* tanh_w;     // device scalar
    double* ld_part;         // [B][gridDim.x] or null
    int H, W, D, mask, mask_c, hc, wc, dc1, dc2, dir;
    // tap mode (tc[0] != null): s_pre / t are the 3x3 conv_out finished here from the tap GEMM
    // C[img][p][(tap, o)] (row stride 9*dc2) of each net, plus bias, and also written to
    // so_w[net] (the raw conv_out the training path reads)
    const float* tc[2];
    const float* tbias[2];
    float* so_w[2];
};

// Whole s,t network of one coupling layer in LDS (cnf_netlds.hip); grid (B, 2 nets).
constexpr int NETLDS_MAXBR = 8;
#ifndef CNF_NETLDS_OTAB
#define CNF_NETLDS_OTAB 192
#endif
constexpr int NETLDS_OTAB = CNF_NETLDS_OTAB;   // byte offset of the parameter-offset table (after the LN slots)
// one conv of k_net_lds: packed format (PK_*), image floats, K extent (PK_KN: padded K; PK_Q4:
// 16 * groups), B row stride (PK_KN)
struct LdsConv {
    int fmt, size, kpad, ns;
};

// A coupling law left pending by the previous layer (forward only): k_net_lds of layer k+1 applies
// layer k's affine law itself (conv_cINN_make_model.py:1215-1233, 1258-1328) — on the fly in its u1c
// gather, and for the whole v_k (split between its two workgroups) with layer k's log-det partials —
// so layer k needs no k_coupling launch. Same arithmetic as k_coupling, element for element.
struct CoupPend {
    const float* u = nullptr;       // u_k [B][H][W][D] (layer k's input; H, W, D as layer k+1's)
    const float* s_pre = nullptr;   // layer k's raw net-A conv_out (pre-tanh) [B][hc][wc][dc2]
    const float* t = nullptr;       // layer k's net-b conv_out
    const float* tanh_w = nullptr;  // layer k's tanh scale
    float* v = nullptr;             // v_k (== layer k+1's u)
    double* ld_part = nullptr;      // layer k's log-det partial slots [B][np]
    int mask_c = 0, hc = 0, wc = 0, dc2 = 0, np = 0, on = 0;
    // comp: layer k+1 conditions on exactly layer k's transformed half (mask_{k+1} == layer k's
    // complement mask, same compressed layout): its u1c gather then yields that half of v_k as is
    // (net A's workgroup stores it with the log-det sum), and net b's copies the other half (layer
    // k's conditioning half, mask / dc1) from u_k — no pass over v_k at the end of the kernel
    int comp = 0, mask = 0, dc1 = 0;
    int W = 0, D = 0;   // u_k's width and depth (k_map2 applies a pending coupling of the last layer of a block)
    // +1: the forward law v2 = exp(s) u2 + t (ld_part collects layer k's sum of s); -1: the inverse
    // law u2 = (1 / exp(s)) (v2 - t) of cnf_flow_inverse (ld_part null). In the inverse schedule
    // "layer k" is the layer just run and "k+1" the one before it in index order, run next.
    int dir = 1;
};

// fp32 constants of the reference's logit map (preprocess_dataset_class, conv_cINN_base_functions.py
// :174-231; TF evaluates the Python-float constants in fp32): c1 = (1-a) b, lo = logit(a),
// span = logit(1-a) - logit(a), inv_bc = 1 / (b (1 - a)) (cnf_transforms.hip logit_consts)
struct LogitK {
    float a, c1, lo, span, inv_bc;
};
// the flow's input as the reference pipeline builds it from the raw xy (conv_cINN.py:246-315): the
// logit map on the x channels (ch < x_d, logit != 0), then instance noise alpha v + (1 - alpha) N(0,1)
// on every channel (cnf_device.h input_prep_value)
struct InputPrepArgs {
    const float* src;   // the raw xy (null: no preparation)
    float alpha;
    unsigned long long seed, off;
    int logit, x_d, D;
    LogitK lk;
};

LogitK logit_consts(float a);   // cnf_transforms.hip
void launch_input_prep(float* out, long long n, const InputPrepArgs& q, hipStream_t st);   // k_prep

struct NetLdsArgs {
    const float* u;           // layer input [B][H][W][D]
    float* so[2];             // outputs: raw conv_out of net A (pre-tanh) / net b, [B][hc][wc][dc2]
    const float* params;      // canonical parameters
    const float* aux;         // dense grouped-conv image
    const int* offs;          // [2][offs_per_net] parameter offsets (see k_net_lds)
    int offs_per_net;
    int H, W, D, mask, hc, wc, dc1, dc2, nk, gc, R, nbr, ln;
    int br_cin_off[NETLDS_MAXBR], br_cin[NETLDS_MAXBR], br_cout[NETLDS_MAXBR], br_out_off[NETLDS_MAXBR],
        br_dil[NETLDS_MAXBR];
    int nwin, win_off[NETLDS_MAXBR], win_len[NETLDS_MAXBR];  // disjoint union of the branch input windows
    int sy, s1, s2, su;                          // LDS pixel strides (floats)
    LdsConv ci, ca, cb, co, gcv[NETLDS_MAXBR];   // packed images of conv_in, conv_a, conv_b, conv_out, branches
    const float* zero_bias;                      // >= 128 zeros (tap GEMM has no bias)
    int off_y, off_t1, off_t2, off_w, off_k;     // LDS byte offsets
    int off_ks;                                  // K-split partial buffers (0: the image has > 4 subtiles)
    int maxnr;                                   // widest conv's 16-column output blocks (picks the instantiation)
    int stamp_off;                               // diagnostic stamp builds: LDS byte offset of the stamp array
    CoupPend pend;                               // previous layer's deferred coupling (pend.on)
    int ci_off[2];                               // conv_in image offset in aux per net (offs[net][0]): its
                                                 // prefetch starts before the offset table is staged
    // training forward (cnf_flow_forward_train): the raw activations and LN statistics the fused
    // backward (k_lds_bwd) reads, one LdsSave block of save_img floats per (net, image), [net][B]
    // (null: inference)
    float* save;
    int save_img, save_t1, save_t2, save_st;
    // fused input preparation (cnf_flow_forward_noise, first coupling only): the u1c gather reads
    // nz.src and applies input_prep_value (logit on the x channels, instance noise of stream element
    // nz.off + flat batch index), and u (then the prepared xy, written here) receives every element
    // of the image: net A's workgroup the gathered half, net b's the transformed half. nz.src null:
    // u is read as is
    InputPrepArgs nz;
};

// Block of one (net, image) in a k_net_lds layer's training save area (all float offsets):
//   y_r  [HW][nk] at r * HW * nk                 (r = 0..R: conv_in's output, then each block's output)
//   t1_r [HW][nk] at t1 + r * HW * nk            (conv_a's raw output)
//   t2_r [HW][gc] at t2 + r * HW * gc            (the grouped stage's raw concat)
//   (mean, rstd) at st: LN1_r at 2r, LN2_r at 2(R + r), LN3_r at 2(2R + r), LN_out at 6R
struct LdsSave {
    int img = 0, t1 = 0, t2 = 0, st = 0;
    static LdsSave of(int HW, int nk, int gc, int R) {
        LdsSave s;
        s.t1 = (R + 1) * HW * nk;
        s.t2 = s.t1 + R * HW * nk;
        s.st = s.t2 + R * HW * gc;
        s.img = (s.st + 2 * (3 * R + 1) + 3) / 4 * 4;
        return s;
    }
};
// The launch-independent "shape" of a k_net_lds launch as int words: [offs_per_net, zero_bias) and
// [off_y, stamp_off) of NetLdsArgs (the mask word inside is not part of it). Shape-specialised
// instantiations take these words as compile-time constants (cnf_netlds_shapes.inc).
constexpr int NETSHAPE_W1 = (int)((offsetof(NetLdsArgs, zero_bias) - offsetof(NetLdsArgs, offs_per_net)) / 4);
constexpr int NETSHAPE_W2 = (int)((offsetof(NetLdsArgs, stamp_off) - offsetof(NetLdsArgs, off_y)) / 4);
constexpr int NETSHAPE_WORDS = NETSHAPE_W1 + NETSHAPE_W2;
static_assert(offsetof(NetLdsArgs, gcv) + sizeof(LdsConv) * NETLDS_MAXBR - offsetof(NetLdsArgs, offs_per_net) == 4 * 123,
              "gen_netlds_shapes.py assumes 123 int members in [offs_per_net, zero_bias)");
constexpr int NETSHAPE_MASK = (int)((offsetof(NetLdsArgs, mask) - offsetof(NetLdsArgs, offs_per_net)) / 4);
inline void netshape_words(const NetLdsArgs& a, int* w) {
    const int* p1 = &a.offs_per_net;
    const int* p2 = &a.off_y;
    for (int i = 0; i < NETSHAPE_W1; i++) w[i] = p1[i];
    for (int i = 0; i < NETSHAPE_W2; i++) w[NETSHAPE_W1 + i] = p2[i];
    w[NETSHAPE_MASK] = 0;
}
// k_gc (cnf_stream.hip): every grouped dilated branch of one residual block for a tile of TH
// image rows of one net, `ipw` images per workgroup. Branch input windows are staged into LDS
// bands with their own dilation halo (LN2 + LeakyReLU applied on the way in, zero padding), so
// the 3x3 taps need no bounds checks; weights are PK_Q4 over cin padded to a multiple of 4.
constexpr int GC_MAXBR = 8;
// waves per k_gc workgroup (one LN partial slot per wave): the shape-specialised instantiations run
// 16 (one 16-pixel subtile per wave and pass, 4 waves per SIMD within 128 VGPRs; 8 waves with two
// subtiles sharing every weight read measured slower with the bf16x6 contraction: 26.2 -> 29.7 us at
// cfg2), small polyphase groups 4-wave workgroups, four per CU; the generic one 8 (two subtiles per wave)
constexpr int GC_NW_GEN = 8, GC_NW_SPEC = 16, GC_NW_MAX = 16;
constexpr int GC_STAGE_QUADS = 2048;   // staged band units per workgroup (2 per thread at 16 waves)
// LDS budget and staged band units of a k_gc workgroup of nw waves (1 workgroup per CU at >= 8 waves,
// 4 at 4)
constexpr int gc_lds_budget(int nw) { return nw >= 8 ? 160 * 1024 : 40 * 1024; }
constexpr int gc_stage_units(int nw) { return nw >= 8 ? 2048 : 2 * 64 * nw; }
constexpr int gc_wg_per_cu(int nw) { return nw >= 8 ? 1 : 4; }
struct GcBranch {
    int cin_off, cin, cinp, cout, out_off, dil;   // input window (cin_off: floats from the image start to pixel 0's window), padded channels, outputs
    int G;                                        // quad groups of the PK_Q4 image
    int band_off, BW, BH, S;                      // LDS band: byte offset, width, height, pixel stride
    int w_off, q_off, b_off;                      // LDS byte offsets: packed weights, quad offsets, bias
    int pcs;                                      // pixel stride of the input window (floats)
    int opcs;                                     // pixel stride of the output slice (out_off: floats from the image start to pixel 0's slice)
    uint32_t cpq_mag, bw_mag;                     // x / (cinp/4) == umulhi(x, cpq_mag) (cinp > 4), x / BW likewise
};
struct GcShape {
    GcBranch br[GC_MAXBR];
    int nbr, H, W, in_cs, out_cs, TH, tiles_per_img;
    int TW, tiles_x;             // tile width (W, or a divisor of W for wide images) and column tiles
    int band_bytes;              // offset of the second band buffer (double-buffered staging)
    int lnst;                    // bit 0: LN2 on load (in_part set), bit 1: LN3 partials out (out_part set)
    // polyphase tiles (ps > 1, one branch of dilation ps): the image splits into ps*ps phase grids
    // (pixels a + i*ps, b + j*ps) of (H/ps) x (W/ps), on which the dilated conv is a dilation-1 conv;
    // a tile is nbk whole phase grids (TH x TW each, nbk > 1) or a TH-row slice of one (tpp slices per
    // grid), its band one (TH+2) x (TW+2) block per grid: the halo of the dilation no longer scales
    // with ps
    int ps, nbk, tpp;
    int nw;                      // waves per workgroup of the shape-specialised instantiation (16, or 4 for
                                 // small bands: four workgroups per CU hide each other's per-image latency)
    int pd;                      // images whose band quads are in flight (registers) ahead of the one computed
};
constexpr int GCSHAPE_WORDS = (int)(sizeof(GcShape) / 4);
struct GcArgs {
    const float* in[2];          // t1 per net [B][HW][in_cs]
    float* out[2];               // t2 per net [B][HW][out_cs]
    const float* in_part[2];     // LN2 partials of t1 (null: no LN)
    float* out_part[2];          // LN3 partials of LeakyReLU(t2)
    const float* gamma[2];       // LN2 gamma/beta [HW][in_cs]
    const float* beta[2];
    const float* w[2][GC_MAXBR];   // per k_gc branch (GcShape.br order)
    const float* b[2][GC_MAXBR];
    GcShape s;                   // launch-independent part (compile-time in the shape-specialised kernels)
    int B, ipw, in_nparts, part_stride;
};
void launch_gc(const GcArgs& a, int grid_x, int lds, hipStream_t st);
int gc_waves(const GcArgs& a);   // waves per workgroup of the instantiation launch_gc picks for a
int read_gc_stamps(long long* host, int n);
int gc_num_shapes();   // shape-specialised k_gc instantiations compiled in
// k_toy (cnf_toy.hip): TOYcINN dense flow, one thread per 3-dimensional sample
constexpr int TOY_MAXL = 128;
struct ToyArgs {
    const float* params;   // canonical flat parameters (per network j: b-block then A-block)
    const float* u;        // [B][3]
    float* v;              // [B][3]
    float* log_detJ;       // [B] (direction -1) or null
    float* per_sample;     // [B][3] (llz, lly, log_detJ) of log_loss (direction -1) or null
    int B, nl, H, L, x_d, dir;
    float lambda_y;
    int order[TOY_MAXL];        // mask_indices
    int net_off[TOY_MAXL + 1];  // float offset of network j's parameters
};
void launch_toy(const ToyArgs& a, int lds_floats, hipStream_t st);
void launch_nll_sums(const float* per_image, float* sums, int B, hipStream_t st);
void launch_net_lds(const NetLdsArgs& a, int B, int lds, hipStream_t st);
int netlds_num_shapes();   // shape-specialised k_net_lds instantiations compiled in
int read_stamps(long long* host, int n);
int read_cycles(long long* host, int n);

void launch_conv(int ks, int mr, int role, const ConvArgs& a, int grid_x, int lds, hipStream_t st);
void launch_conv1(int mr, bool vec, int role, const ConvArgs& a, int grid_x, int lds, hipStream_t st);
// k_pw launch shape: every launch-independent field a shape-specialised k_pw instantiation folds
// in (cnf_stream.hip; table generated by gen_netlds_shapes.py from a dry run of the forward)
struct PwShape {
    int nr, gm, ln, res, tap;            // template selection
    int H, W, tiles_per_img, nprob;
    int in_cs, in_off, cin, out_cs, out_off, cout, lds_w_off, part_stride;
    int umask, uW, uD, udc, uimg, udil, uoff;   // tap mode (0 otherwise)
    uint32_t st_mask_lo, st_mask_hi;
    int st_compact, in_mapped;
};
constexpr int PWSHAPE_WORDS = (int)(sizeof(PwShape) / 4);
// the shape of a k_pw launch; false when its problems differ in a shape field
inline bool pw_shape_of(int nr, int gm, bool ln, bool res, bool tap, const ConvArgs& a, PwShape& s) {
    const ConvProb& q = a.p[0];
    s = PwShape{nr, gm, ln ? 1 : 0, res ? 1 : 0, tap ? 1 : 0, a.H, a.W, a.tiles_per_img, a.nprob, q.in_cs, q.in_off,
                q.cin, q.out_cs, q.out_off, q.cout, q.lds_w_off, q.part_stride,
                tap ? a.umask : 0, tap ? a.uW : 0, tap ? a.uD : 0, tap ? a.udc : 0, tap ? a.uimg : 0,
                tap ? a.udil : 0, tap ? a.uoff : 0,
                q.st_mask_lo, q.st_mask_hi, q.st_compact, q.in_mapped};
    for (int i = 1; i < a.nprob; i++) {
        const ConvProb& r = a.p[i];
        if (r.in_cs != q.in_cs || r.in_off != q.in_off || r.cin != q.cin || r.out_cs != q.out_cs ||
            r.out_off != q.out_off || r.cout != q.cout || r.lds_w_off != q.lds_w_off || r.part_stride != q.part_stride ||
            r.st_mask_lo != q.st_mask_lo || r.st_mask_hi != q.st_mask_hi || r.st_compact != q.st_compact ||
            r.in_mapped != q.in_mapped)
            return false;
    }
    return true;
}
void launch_pw(int nr, int gm, bool ln, bool res, bool tap, const ConvArgs& a, int grid_x, int lds, hipStream_t st);
int pw_num_shapes();
int read_pw_stamps(long long* host);   // diagnostic builds (CNF_PW_STAMPS=SID): [2048 workgroups][12]
void launch_convtap(int mt, bool vec, const ConvArgs& a, int grid_x, int lds, hipStream_t st);
void launch_gather_u1c(const float* u, float* u1c, int B, int H, int W, int D, int mask, int hc, int wc, int dc1,
                       hipStream_t st);
void launch_coupling(const CoupArgs& a, int B, int nparts, hipStream_t st);
void launch_ld_reduce(const double* part, float* out, int B, int nl, int np, int accumulate, hipStream_t st);
// LN partial slots [B][part_stride][LNP] of one tensor (two nets: part0, part1 or null) merged into
// slot 0 of each image (k_ln_merge): consumers then read nparts = 1
void launch_ln_merge(float* part0, float* part1, int nparts, int part_stride, int B, hipStream_t st);
// (mean, rstd) [B][2] per net of up to LNF_MAX LN tensors from their producers' partial slots (as in_ln),
// one launch: tensor i's slots part[i][net] ([B][part_stride][LNP], nparts[i] used) -> st[i][net]
constexpr int LNF_MAX = 4;
struct LnFinalSet {
    const float* part[LNF_MAX][2];
    float* st[LNF_MAX][2];
    int nparts[LNF_MAX];
    int count, part_stride;
};
void launch_ln_final(const LnFinalSet& s, int B, hipStream_t st);
void launch_map_gather(const float* src, float* dst, const int* idx, int n, int ss, int ds, int B, hipStream_t st);
void launch_map_scatter(const float* src, float* dst, const int* sidx, const int* didx, int n, int ss, int ds,
                        int B, hipStream_t st);
// two independent index maps (+ optionally the per-image log-det reduction) in one launch:
// dst[b, didx ? didx[i] : i] = src[b, sidx ? sidx[i] : i] (a gather has didx == null, a scatter sidx
// == null or a source map). The forward's factor boundaries (keep gather + factored scatter) and its
// tail (final scatter + log-det reduction) each take one launch instead of two.
struct MapOp {
    const float* src = nullptr;
    float* dst = nullptr;
    const int* sidx = nullptr;
    const int* didx = nullptr;
    int n = 0, ss = 0, ds = 0;
    int pend = 0;   // k_map2: read the source through the launch's pending coupling (src is then unused)
};
struct LdReduce {
    const double* part = nullptr;   // null: no reduction
    float* out = nullptr;
    int nl = 0, np = 0, accumulate = 0;
};
// pend.on: the maps read v_k of a deferred coupling (computed from u_k, s, t on the fly; src is
// unused), and the extra block computes layer k's log-det sum — into its partial slots, or, with
// r.part, straight into the per-image total (r.nl then counts the layers before k)
void launch_map2(const MapOp& a, const MapOp& b, const LdReduce& r, const CoupPend& pend, int B, hipStream_t st);
void launch_squeeze(const float* in, float* out, int B, int H, int W, int C, int dir, hipStream_t st);
void launch_chcopy(const float* in, int in_cs, int in_off, float* out, int out_cs, int out_off, int C, long long npix,
                   hipStream_t st);
// per-image NLL terms and the batch sums in one launch; done: a zero-initialised device counter
// owned by the caller, left at 0 by every completed launch (concurrent launches need their own)
void launch_nll(const float* xy, const float* zy, const float* ld, float* per_image, float* sums, unsigned* done,
                int B, int HW, int D, int x_d, float lambda_y, hipStream_t st);
void launch_pack(const float* params, const int64_t* map, float* aux, long long n, hipStream_t st);


// ---- training (cnf_train.hip) -------------------------------------------------------------------
// Generic fp32 convolution for the training path over the dense backward image (taps x k x n):
//   out[b,p,n] (=|+=) bias[n] + res[b,p,n] + sum_{tap,k} X[b, p + sgn*dil*off(tap), k] * W(tap,k,n)
// with W(tap,k,n) = w[tap*wt + k*wk + n*wn] and X = LN(LeakyReLU(in)) on load when stats != null
// (LeakyReLU only when act && !stats). sgn = +1 is the forward conv; sgn = -1 with transposed
// strides is the data gradient (dX = conv^T dY). Zero padding outside the image.
struct TConvArgs {
    const float* in;
    int in_cs, in_off, K;
    const float* stats;       // [B][2] (mean, rstd) of LeakyReLU(in) over the whole tensor, or null
    const float* gamma;       // per element [npx][in_cs] (channel in_off + k)
    const float* beta;
    int act;
    const float* w;
    long long wt;
    int wk, wn;
    const float* bias;        // [N] or null
    const float* res;         // [B][npx][out_cs] window or null
    float* out;
    int out_cs, out_off, N, accumulate;
    int H, W, taps, dil, sgn, B;
    const float* zero;        // >= 16 bytes of zeros, 16-byte aligned: what out-of-image loads read
    // LN-backward reduction of the output (lnr_part non-null): the output v is dL/d(LN output) of the
    // LayerNorm(LeakyReLU) whose raw input lnr_x has the output's layout; each workgroup adds sum v * gamma
    // and sum v * gamma * xhat over its elements and writes them to lnr_part[b][tile][2] (fixed order)
    const float* lnr_x;
    const float* lnr_gamma;
    const float* lnr_stats;
    double* lnr_part;
    int lnr_base, lnr_stride;   // the launch's partials at [b][lnr_base + tile] of a [B][lnr_stride] array
};
// returns the LN-reduction partials per image the launch wrote (0: none — the kernel has no fused
// reduction, the caller runs k_lnb_reduce)
int launch_tconv(const TConvArgs& a, hipStream_t st);
constexpr int LNR_MAXPARTS = 64;   // per image, k_tconv_* fused LN reductions

// weight gradient: part[chunk][(tap*CI + ci)*CO + co] = sum over the chunk's pixels of
// X[b, p + dil*off(tap), ci] * dY[b, p, co] (X with LN-on-load as in TConvArgs); bpart[chunk][co]
// = sum dY (bias gradient) when non-null
struct WGradArgs {
    const float* x;
    int x_cs, x_off, CI;
    const float* stats;
    const float* gamma;
    const float* beta;
    int act;
    const float* dy;
    int dy_cs, dy_off, CO;
    float* part;
    float* bpart;
    int H, W, taps, dil, B, chunks, chunk_px;
    const float* zero;   // k_wgrad_direct: >= 1 float of zeros (what lanes outside the image read)
};
void launch_wgrad(const WGradArgs& a, hipStream_t st);
// k_wgrad_band (the MFMA weight gradient): partial rows per launch (<= WGRAD_MAX_CHUNKS), each
// [taps][CI][CO] weights then [CO] bias, and its LDS bytes
constexpr int WGRAD_MAX_CHUNKS = 256;
int wgrad_band_chunks(int B, int H, int W, int taps, int CI, int CO);
size_t wgrad_band_lds(int H, int W, int taps, int dil, int CI, int CO);
bool train_valu_kernels();   // CNF_TRAIN_VALU=1: the register-blocked VALU convolutions (A/B)
// k_wgrad_band handles this conv (taps 1 / 9, width >= 4, staged band within 160 KiB); otherwise the
// weight gradient runs on the VALU k_wgrad (WGradArgs::chunk_px > 0) with a separate bias scatter
bool wgrad_band_ok(int H, int W, int taps, int dil, int CI, int CO);
// k_wgrad_direct (register-operand MFMA weight gradient, WGradArgs::chunk_px == -1): width % 4 == 0,
// taps 1 / 9; its partial-row count (<= WGRAD_MAX_CHUNKS) for a batch of B images of H rows
bool wgrad_direct_ok(int H, int W, int taps);
int wgrad_direct_chunks(int B, int H);
// k_wgrad_thin (3x3, dilation 1, CO <= 4, CI <= 64, CI % 4 == 0: the streamed conv_out's weight
// gradient): one partial row [taps][CI][CO] + [CO] per workgroup, wgrad_thin_chunks of them
bool wgrad_thin_ok(int H, int W, int taps, int dil, int CI, int CO);
int wgrad_thin_chunks(int B, int H, int W);
void launch_wgrad_thin(const WGradArgs& a, hipStream_t st);
// dparams[map[i]] += sum_c part[c][i] for i < n (map[i] >= 0)
void launch_grad_scatter(const float* part, int chunks, long long n, const int64_t* map, float* dparams, hipStream_t st);
void launch_ln_stats(const float* x, long long n, int B, int act, float* stats, hipStream_t st);
// LN + LeakyReLU backward: dx (=|+=) d/dx of LN(LeakyReLU(x)) given dxo = dL/d(LN output);
// dgamma/dbeta (+=) per element; stats == null: LeakyReLU backward only
// (the batch runs in LNB_SLICES slices: scratch holds their [2][LNB_SLICES][n] gamma / beta partials)
constexpr int LNB_SLICES = 8;
// k_lnb_reduce splits each image over up to LNB_RS workgroups (partial sums [B][rs][2], summed in slice
// order where they are read)
constexpr int LNB_RS = 8;
// presum > 0: sums already holds presum partials per image at [b][k] of a [B][pstride][2] array (k_tconv_*
// fused LN reductions), no k_lnb_reduce. cmod > 0: dxo holds only the channels whose bit is set in
// cmask (channel = element index % cmod, cmod <= 64); the others are read as 0 whatever dxo holds
void launch_ln_backward(const float* x, const float* dxo, const float* gamma, const float* stats, double* sums,
                        long long n, int B, int act, float* dx, int accumulate, float* dgamma, float* dbeta,
                        float* scratch, hipStream_t st, int presum = 0, int pstride = 0,
                        unsigned long long cmask = 0, int cmod = 0);
// Fused training backward of a k_net_lds layer (cnf_ldsbwd.hip): grid (B, 2 nets), one workgroup per
// (image, net). Offsets table per net (int32, `offs_per_net` entries): canonical parameter offsets
// (LN gamma / beta, the net's first parameter, tanh scale or -1) and dense backward-image offsets
// (conv weights _DW, biases _DB), laid out as the LDSBWD_* indices below (per residual block r at
// LDSBWD_RB0 + r * (LDSBWD_PER_RB0 + 2 * nbr), branch bi's (dw, db) at LDSBWD_BR + 2 bi of it).
enum {
    LDSBWD_LO = 0, LDSBWD_CI_DW, LDSBWD_CI_DB, LDSBWD_LNO_G, LDSBWD_LNO_B, LDSBWD_CO_DW, LDSBWD_CO_DB, LDSBWD_TANH,
    LDSBWD_CI_K, LDSBWD_CI_B, LDSBWD_CO_K, LDSBWD_CO_B,   // canonical kernel / bias offsets of the plain convs
    LDSBWD_RB0
};
enum {
    LDSBWD_LN1G = 0, LDSBWD_LN1B, LDSBWD_CA_DW, LDSBWD_CA_DB, LDSBWD_LN2G, LDSBWD_LN2B, LDSBWD_LN3G, LDSBWD_LN3B,
    LDSBWD_CB_DW, LDSBWD_CB_DB, LDSBWD_CA_K, LDSBWD_CA_B, LDSBWD_CB_K, LDSBWD_CB_B, LDSBWD_BR
};
constexpr int LDSBWD_PER_RB0 = LDSBWD_BR;   // entries per residual block before its branches' (dw, db) pairs
struct LdsBwdArgs {
    const float* save;        // the training forward's save area of the layer [net][B][save_img] (LdsSave)
    int save_img, save_t1, save_t2, save_st;
    const float* dso[2];      // dL/d(raw conv_out) per net [B][hc][wc][dc2] (k_coup_bw)
    const float* u;           // the layer input [B][H][W][D] (conv_in reads its mask-compressed half)
    float* du1c[2];           // out: dL/du1c per net [B][hc][wc][dc1]
    const float* params;      // canonical parameters (LN gamma / beta)
    const float* bw;          // dense backward weight image (launch_pack)
    const int64_t* bw_map;    // dense -> canonical parameter index
    const int* offs;          // [2][offs_per_net]
    int offs_per_net;
    float* part;              // out: per (net, image) gradient rows [2][B][row], the net's canonical range
    int row;
    int H, W, D, mask, hc, wc, dc1, dc2, nk, gc, R, nbr, ln, taps;
    int br_cin_off[NETLDS_MAXBR], br_cin[NETLDS_MAXBR], br_cout[NETLDS_MAXBR], br_out_off[NETLDS_MAXBR],
        br_dil[NETLDS_MAXBR];
    int sy, st, sa, ac_chunk;                                   // LDS pixel strides (floats); conv_b staging chunk
    int wmax;                                                   // floats of the W region (weight-gradient scratch too)
    int stamps;                                                 // diagnostics: phase clock stamps (CNF_LDSBWD_STAMPS)
    int off_gt, off_ac, off_w, off_kt, off_red, off_ot, off_z, lds_bytes;   // LDS byte offsets (GY at 0)
    // split mode (CNF_LDS_SPLIT): 0 the whole backward; 1 the data-gradient chain only, storing the
    // gradients the weight gradients contract with to gsave; 2 the weight gradients only, from gsave
    int mode;
    float* gsave;                       // [2][B][gsave_img] per (net, image)
    int gsave_img, gs_rb, g_t3, g_t2, g_in;   // per residual block r: dL/dy_{r+1} at r * gs_rb, dL/dt2 at
                                             // + g_t3, dL/dt1 at + g_t2; dL/dy_0 (conv_in's) at g_in
};
void launch_lds_bwd(const LdsBwdArgs& a, int B, hipStream_t st);
int read_bwd_stamps(long long* host, int n);   // [0] = count, [1..] = s_memtime per phase boundary
// dparams[lo_n + i] += sum_b part[n][b][i] (i < len_n, n = 0, 1; row floats per (net, image) row)
void launch_grad_rows(const float* part, int B, int row, int64_t lo0, int64_t lo1, int len0, int len1, float* dparams,
                      hipStream_t st);

struct CoupBwArgs {
    const float* u;           // layer input [B][H][W][D]
    const float* dv;          // dL/dv
    const float* s_pre;       // raw conv_out of net A
    const float* tanh_w;
    float* du;                // dL/du (u1 positions: dL/dv1 only; the nets' share is added later)
    float* ds_pre;            // dL/d s_pre  [B][hc][wc][dc2]
    float* dt;                // dL/dt
    double* dw_part;          // [B][gridDim.x]
    float g_ld;               // dL/d(per-image log-det)
    const float* count;       // non-null: g_ld = -1 / *count (the global image count, on device)
    int H, W, D, mask, mask_c, hc, wc, dc1, dc2;
};
void launch_coupling_backward(const CoupBwArgs& a, int B, int nparts, hipStream_t st);
void launch_scatter_add_u1c(const float* du1c, float* du, int B, int H, int W, int D, int mask, int hc, int wc, int dc1,
                            hipStream_t st);
void launch_dsum(const double* part, long long n, float* out, hipStream_t st);
// dL/dzy of the NLL (conv_cINN_make_model.py:1800-1848): z / Bg, lambda_y * sign(y - y') / Bg
// count (device, may be null): the global image count; when given, inv_batch = 1 / *count (computed in
// fp64 and rounded once, as the host does), so the scale needs no host read of the all-reduced count
void launch_nll_grad(const float* xy, const float* zy, float* dzy, int B, int HW, int D, int x_d, float lambda_y,
                     float inv_batch, const float* count, hipStream_t st);
void launch_adam(float* params, const float* grads, float* m, float* v, long long n, float alpha, float b1, float b2,
                 float eps, hipStream_t st);
}  // namespace cnf
