// cnf_plan.h — host-side model plan: the cFlow schedule (conv_cINN_make_model.py:1431-1695),
// the canonical parameter table, the dense grouped-conv aux image, the squeeze/factor index maps
// and the workspace layout. No GPU code here.
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>
#include <functional>
#include <string>
#include <memory>
#include <mutex>
#include <vector>

#include "../../include/cnf.h"
#include "cnf_kernels.h"

namespace cnf {

struct Branch {
    int dil = 1;              // dilation factor of the branch (base_functions.py:575-601)
    int width = 0;            // _d = int((nk // d) // card)   (base_functions.py:397)
    int out_off = 0;          // channel offset inside the concat
    std::vector<int> in_offsets;  // per group: first input channel read (closure quirk aware)
    // dense-conv view used by the kernels: 3x3 conv from channels [cin_off, cin_off+cin)
    int cin_off = 0, cin = 0, cout = 0;
};

// A convolution's weights + bias as packed into the device "kernel image" (the aux buffer) in the
// exact LDS layout its kernel consumes, so staging is a plain float4 copy:
//   PK_1X1  1x1 conv [cin][cout]: B image [g][q][j][s], element (c = 16g+4q+s, j), j < 16*nr
//   PK_TAP  3x3 conv as tap GEMM: same image over c with columns j = tap*cout + o (9*cout <= 64)
//   PK_KN   3x3 implicit GEMM: [kpad][ns], k = tap*cin + c, ns = 16*nr (+16 if ns % 32 == 0)
//   PK_Q4   3x3 as a list of channel quads qd = tap*(cin/4) + cq: [g][q][j][s], qd = 4g + q,
//           k = tap*cin + 4cq + s (cin % 4 == 0; LDS kernel: one ds_read_b128 per quad)
// (the PK_* constants live in cnf_kernels.h, shared with the kernels)
struct PackedConv {
    int fmt = PK_KN, cin = 0, cout = 0, nr = 0, ns = 0, G = 0, kpad = 0;
    int64_t w = -1, b = -1, size = 0;   // offsets (floats) into the kernel image; size of the weight image
    // training: offsets into the dense backward image (bw image): [taps][cin][cout] weights, [cout] bias
    int64_t dw = -1, db = -1;
    int taps = 9;
};

struct RBParams {
    int64_t ln1g = -1, ln1b = -1, conv_a_k = -1, conv_a_b = -1, ln2g = -1, ln2b = -1;
    std::vector<std::vector<int64_t>> gk, gb;  // [branch][group] canonical offsets
    int64_t ln3g = -1, ln3b = -1, conv_b_k = -1, conv_b_b = -1;
    PackedConv ca, cb;                         // conv_a, conv_b (PK_1X1)
    std::vector<PackedConv> gc;                // grouped branches as dense 3x3 convs (PK_KN)
    std::vector<PackedConv> gpw;               // streamed, k_gc not fused: branch as a 1x1 over its 9*cin im2col row (size 0: none)
    int64_t ln2c_g = -1, ln2c_b = -1;          // aux: LN2 gamma/beta gathered to the compact t1 layout (t1_compact)
    int64_t ln3c_g = -1, ln3c_b = -1;          // aux: LN3 gamma/beta in the mapped t2 layout (t2_mapped)
};

struct NetParams {
    int64_t conv_in_k = -1, conv_in_b = -1;
    std::vector<RBParams> rb;
    int64_t ln_out_g = -1, ln_out_b = -1, conv_out_k = -1, conv_out_b = -1, tanh_w = -1;
    PackedConv ci, co;                         // conv_in (PK_KN), conv_out (PK_TAP or PK_KN)
    int64_t lo = -1, hi = -1;                  // the net's canonical parameter range [lo, hi)
    PackedConv ci_pw;                          // streamed conv_in as a 1x1 over its 9*dc1 im2col row (PK_1X1; size 0: none)
    std::vector<PackedConv> co_chunks;         // streamed conv_out with > 64 outputs: 64-column PK_KN chunks
};

// LDS image of k_net_lds (cnf_netlds.hip): Y | T1 | T2 | W | K, byte offsets; pixel strides in floats
struct NetLdsGeom {
    int sy = 0, s1 = 0, s2 = 0, su = 0, s2r = 0;
    int off_y = 0, off_t1 = 0, off_t2 = 0, off_w = 0, off_k = 0, bytes = 0;
    int off_ks = 0;   // images of at most 4 subtiles: K-split partial sums (0 = none)
};

struct Coupling {
    int index = 0, block = 0, H = 0, W = 0, D = 0, mask = 0, mask_c = 0;
    int hc = 0, wc = 0, dc1 = 0, dc2 = 0, nk = 0, card = 0, R = 0;
    std::vector<int> dils;
    std::vector<Branch> br;
    int gc = 0;               // concat width of the grouped stage
    NetParams net[2];         // 0 = A (scale), 1 = b (translation)
    // k_net_lds parameter-offset table: [net][conv_in_k, conv_in_b, per rb (ln1g, ln1b, conv_a_k,
    // conv_a_b, ln2g, ln2b, ln3g, ln3b, conv_b_k, conv_b_b, aux_w/aux_b per branch), ln_out_g,
    // ln_out_b, conv_out_k, conv_out_b]; offsets into params (aux offsets into the aux image)
    std::vector<int> lds_offs;
    int lds_offs_per_net = 0;
    int dev_lds_offs = -1;    // offset into the device table
    bool use_lds = false;     // run the whole s,t net in one workgroup (k_net_lds)
    int ci_fmt = PK_KN, co_fmt = PK_KN;   // packed formats of conv_in / conv_out
    std::vector<int> gc_fmt;              // per grouped branch
    NetLdsGeom lds;                       // valid when use_lds
    // training: the fused backward of a k_net_lds layer (cnf_ldsbwd.hip) when its LDS image fits
    // (CNF_LDS_BWD=0 at plan creation: the multi-kernel backward); the training forward then saves the
    // layer's raw activations (LdsSave) and s/t outputs for it
    bool lds_bwd = false;
    std::vector<int> bwd_offs;            // [net][bwd_offs_per_net] (LDSBWD_* layout)
    int bwd_offs_per_net = 0;
    int dev_bwd_offs = -1;
    // streamed layer: the grouped stage as k_gc launches (PK_Q4, padded cin), each over a group of
    // branches that fits one workgroup's LDS; branches in none run as k_pw tap-mode launches (k_conv<3>
    // when their im2col row is too long)
    struct GcGroup {
        std::vector<int> br;              // indices into Coupling::br
        std::vector<GcBranch> gcb;        // their geometry (offsets into LDS)
        int TH = 0, TW = 0, tiles_x = 1;  // tile rows / columns (W, or a divisor of W), column tiles
        int lds = 0, band_bytes = 0;      // LDS bytes per workgroup; bytes of one set of branch bands
        int tiles() const { return tiles_y * tiles_x; }
        int tiles_y = 1;
        int TP = 0;                       // tile pixels the plan aimed at (TH = min(H, TP / TW))
        int ps = 1, nbk = 1, tpp = 1;     // polyphase tiles (GcShape): phase stride, grids per tile, slices per grid
        int nw = GC_NW_SPEC;              // waves per workgroup (GcShape::nw)
        int pd = 1;                       // band prefetch depth in images (GcShape::pd)
    };
    std::vector<GcGroup> gcg;
    bool gc_fused = false;                // gcg non-empty
    // streamed layers: t1 (conv_a's output) holds only the channels the grouped branches read, one
    // dense sub-tensor per consumer (a k_gc group, or a branch launched on its own) inside each
    // image: sub-tensor u = [HW][cs_u] at float offset HW * (cs_0 + ... + cs_{u-1}), its windows
    // packed in channel order, each from a 16-byte boundary. t1_cs = floats per pixel of an image (nk when plain),
    // t1_off[bi] / t1_pcs[bi] = branch bi's window: offset of pixel 0 inside the image, pixel
    // stride; t1_map[2c], [2c+1] = the same for channel c (-1: not stored)
    uint64_t t1_used = 0;
    int t1_cs = 0;
    bool t1_compact = false;
    std::vector<int> t1_off, t1_pcs, t1_map;
    int dev_t1_map = -1;   // offset of t1_map in the device table
    // ... and t2 (the grouped stage's concat, conv_b's input) likewise when several launches produce it:
    // one dense sub-tensor per producer, so a k_gc group of a few output channels stores whole lines
    // instead of 16-32 bytes of every (124-channel) pixel. t2_cs = floats per pixel of an image,
    // t2_off[bi] / t2_pcs[bi] = branch bi's output slice (offset of pixel 0, pixel stride), t2_qmap =
    // (offset, stride) per input quad of conv_b, t2_bmap[bi] = branch bi's per-output-channel store map
    bool t2_mapped = false;
    int t2_cs = 0;
    std::vector<int> t2_off, t2_pcs, t2_qmap;
    std::vector<std::vector<int>> t2_bmap;
    int dev_t2_qmap = -1;
    std::vector<int> dev_t2_bmap;
    bool in_gc(int bi) const {
        for (const GcGroup& g : gcg)
            for (int b : g.br)
                if (b == bi) return true;
        return false;
    }
};

struct Layer {
    int kind = CNF_LAYER_COUPLING;
    int ci = -1;              // coupling index
    int npf = 0;              // num_prev_factors (factor layers)
    int h = 0, w = 0, d = 0;  // block io shape
    int block = 0;
};

struct ParamTensor {
    std::string name;
    int64_t offset = 0;
    std::vector<int> shape;
    int64_t size() const {
        int64_t s = 1;
        for (int v : shape) s *= v;
        return s;
    }
};

// Squeeze+factor boundary after a block, as index maps over per-image element
// indices. keep_src[i]: index in the current block layout of element i of the next
// block layout. fac_src[j]/fac_orig[j]: index in current layout / position in the
// final xy-layout output of the j-th factored-out element.
struct Boundary {
    int after_block = 0;
    int n_cur = 0, n_next = 0, n_fac = 0;
    std::vector<int> keep_src, fac_src, fac_orig;
    int dev_keep_src = -1, dev_fac_src = -1, dev_fac_orig = -1;  // offsets into the device table
};

// A recorded kernel launch (for bench measurement hooks).
struct Recorded {
    std::string name;
    double flops = 0, bytes = 0;
    std::function<void(void*)> relaunch;
    bool timed = false;   // its kernel wrote begin / end timestamps into the plan's event pair
};

struct WsLayout {
    size_t total = 0;
    size_t uv[2] = {0, 0}, u1c = 0, y[2] = {0, 0}, t1[2] = {0, 0}, t2[2] = {0, 0}, so[2] = {0, 0};
    size_t so_alt[2] = {0, 0};   // k_net_lds layers of odd index write s/t here (a deferred coupling reads the other set)
    size_t st_part[2][3] = {};   // LN partials [net][y, t1, t2]
    size_t ld = 0;
    int64_t n_uv = 0, n_u1c = 0, n_y = 0, n_t2 = 0, n_so = 0;
    int st_parts = 0;   // partial slots per image per LN slab
    int ld_parts = 0;   // log-det partial slots per image per coupling layer
};

// training workspace (after the inference layout): saved coupling inputs, the dense backward
// weight image, one coupling layer's recomputed activations and the gradient buffers
struct TrainLayout {
    size_t total = 0;
    std::vector<size_t> save_u;   // per coupling index: its input u [B][H][W][D]
    size_t bw = 0;
    size_t ys[2] = {}, t1s[2] = {}, t2s[2] = {}, so[2] = {}, dso[2] = {}, stats[2] = {};
    // per-net scratch ([net]): the two nets' backward chains run on two streams
    size_t dy[2] = {}, dln[2] = {}, dbuf[2] = {}, dt1[2] = {}, dc[2] = {}, dt2[2] = {}, du1c[2] = {};
    size_t u1c = 0, duv[2] = {}, dzy = 0;
    size_t lnsum[2] = {}, wpart[2] = {}, bpart[2] = {}, lnpart[2] = {}, dwpart = 0;
    size_t zeros = 0;   // 64 floats of zeros (k_wgrad_direct's address for loads outside the image)
    // fused LDS-layer backward: per coupling index the forward's save area [2][B][LdsSave::img] and s/t
    // outputs [2][B][hc][wc][dc2] (0: none), and the per-(net, image) gradient rows [2][B][row_max]
    std::vector<size_t> act_save, so_save;
    size_t rows = 0;
    int row_max = 0;
    // split LDS backward (chain and weight gradients as two launches, CNF_LDS_SPLIT): per parity of the LDS
    // layer count a second row set (rows2), the stored chain gradients [2][B][gsave_max] and the coupling
    // gradients dL/d(so) [net]: layer k's weight gradients run behind layer k+1's chain, so their buffers
    // alternate
    size_t rows2 = 0, gsave[2] = {}, dso_l[2][2] = {};
    int gsave_max = 0;
    // streamed layers: the training forward saves the activations the backward would otherwise recompute
    // (when they fit the budget): per net y [R+1][B][HW][nk], full t1 [R][B][HW][nk], t2 [R][B][HW][gc],
    // LN statistics [3R+1][B][2] (y_r: r, t1_r: R+1+r, t2_r: 2R+1+r) and the raw conv_out [2][B][HW][dc2]
    struct StreamSave {
        size_t y[2] = {}, t1[2] = {}, t2[2] = {}, st[2] = {}, so = 0;
    };
    std::vector<StreamSave> ssave;
    std::vector<char> has_ssave;
};

struct Plan {
    cnf_flow_desc desc{};
    std::vector<int> sfbl, rbl, nkl, cl;
    std::vector<Layer> layers;
    std::vector<Coupling> couplings;
    std::vector<ParamTensor> params;
    int64_t n_params = 0;
    int64_t n_aux = 0;
    int64_t aux_zero = 0;           // offset of 128 zero floats in the kernel image
    std::vector<int64_t> aux_map;   // kernel image: aux[i] = params[aux_map[i]] (or 0 if < 0)
    // training: dense backward image bw[i] = params[bw_map[i]] (0 if < 0); the same map scatters
    // dense weight gradients back onto the canonical parameters
    std::vector<int64_t> bw_map;
    int64_t n_bw = 0;
    int64_t* dev_bw_map = nullptr;
    std::vector<Boundary> boundaries;
    std::vector<int> final_orig;    // last block layout -> xy position
    int last_n = 0;                 // elements per image of the last block layout
    // device constant tables (int32), uploaded lazily
    std::vector<int> host_table;
    int* dev_table = nullptr;
    int64_t* dev_aux_map = nullptr;
    int dev_final_orig = -1;
    int device = -1;
    // launch recording
    bool record = true;
    bool dry = false;         // host-only dry run: record launches without issuing them (shape dumps)
    std::vector<PwShape> pw_shapes;   // k_pw launch shapes seen by a dry run
    std::vector<GcShape> gc_launch;   // dry runs: the k_gc launch shapes (GcArgs::s) as run_coupling issues them
    std::vector<std::string> dry_launches;   // dry runs: the launch names in issue order (cnf_debug_schedule)
    Options opts;             // cnf_flow_desc.debug_options (parsed by build_plan)
    bool use_pw = true;       // image-looping k_pw for streamed 1x1 convs (option PW=0: per-tile k_conv1)
    bool tap_pw = true;       // streamed tap conv_out as a 1x1 tap GEMM + sums in k_coupling (PW=0: k_convtap)
    std::vector<Recorded> recorded;
    // in-stream launch timing (bench.py): a HIP event pair around every recorded launch
    bool timing = false;
    std::vector<hipEvent_t> ev;   // 2 per recorded launch, grown on demand, owned by the plan
    // training: net b's recompute / backward chain runs on a second stream (fork / join events)
    hipStream_t side = nullptr;
    hipEvent_t ev_fork = nullptr, ev_join = nullptr;
    int side_device = -1;
    // ... and each net's weight gradients on a stream of their own (wside[net]), ordered against the
    // chain by events from tev (reused once a coupling's streams have joined)
    hipStream_t wside[2] = {nullptr, nullptr};
    std::vector<hipEvent_t> tev;
    size_t tev_next = 0;
    // cnf_nll's completion counters: NLL_SLOTS ints past the device table, one per stream that has
    // called cnf_nll on this plan (host-side assignment, so concurrent calls on different streams
    // never share a counter and a call inside graph capture needs no allocation). A 65th stream takes
    // the least recently used slot behind a wait on that slot's last launch (nll_ev)
    static constexpr int NLL_SLOTS = 64;
    std::vector<void*> nll_streams;
    std::vector<hipEvent_t> nll_ev;
    std::vector<uint64_t> nll_last;
    uint64_t nll_clock = 0;
    std::shared_ptr<std::mutex> nll_mu = std::make_shared<std::mutex>();
    WsLayout layout(int B) const;
    TrainLayout train_layout(int B) const;
    // device-table address of entry `off`; host-only dry runs carry no device tables, so they get a
    // placeholder base (the address is recorded, never dereferenced, and never null + offset)
    const int* dtab(int64_t off) const {
        return (dry ? reinterpret_cast<const int*>(uintptr_t(1) << 40) : dev_table) + off;
    }
};

// cnf_train.cpp: dL/dparams of the NLL (loss scaled by inv_batch = 1 / global batch) into dparams,
// from the coupling inputs saved by the training forward in `workspace`
// fused LDS-layer backward geometry of coupling c (LDS layout, strides, shape fields of a); returns the
// LDS bytes, 0 when it does not fit (cnf_train.cpp)
size_t ldsbwd_setup(const Plan& p, const Coupling& c, LdsBwdArgs& a);
typedef void (*LayerDoneFn)(void* user, int coupling_index);
void flow_backward(Plan& p, const float* params, const float* xy, const float* zy, void* workspace, int B,
                   float inv_batch, float* dparams, hipStream_t st, const float* count = nullptr,
                   LayerDoneFn done = nullptr, void* user = nullptr);
// one coupling layer's backward: du, dparams (zeroed first) for dL/dv = dv and dL/d logdet_b = g_ld
void coupling_layer_backward(Plan& p, int ci, const float* params, const float* u, const float* dv, float* du,
                             float g_ld, void* workspace, int B, float* dparams, hipStream_t st);

// builds the plan; throws std::invalid_argument with the reference's assertion text
Plan* build_plan(const cnf_flow_desc* d);

}  // namespace cnf
