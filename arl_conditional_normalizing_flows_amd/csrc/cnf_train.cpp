// cnf_train.cpp — backward pass of the NLL training step (cFlow.train_step,
// conv_cINN_make_model.py:1850-1880: tf.GradientTape over log_loss :1800-1848).
//
// Gradient of loss = -(mean_b(llz_b + lly_b) + mean_b(logdet_b)) with respect to the canonical
// parameter vector. The forward (cnf_flow_forward_train) saves every coupling layer's input; the
// backward walks the layer schedule in reverse:
//   - layout layers (squeeze / factor-out / final restoration) are permutations: their gradient is
//     the inverse map applied to dL/dv (the same index tables as cnf_flow_inverse);
//   - a coupling layer recomputes both s,t networks from its saved input (activations of every
//     residual block kept for this one layer), runs the coupling-law backward, then each network
//     in reverse: conv weight gradients (k_wgrad + scatter through the dense map onto the
//     canonical parameters, so the grouped-conv closure quirk and group boundaries come out
//     exactly), data gradients (k_tconv with transposed weights), LayerNorm backward with the
//     per-element gamma/beta gradients.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <vector>

#include "cnf_kernels.h"
#include "cnf_plan.h"

namespace cnf {

namespace {

inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }

void hchk(hipError_t e, const char* what) {
    if (e != hipSuccess) throw std::runtime_error(std::string(what) + ": " + hipGetErrorString(e));
}

// LN-on-load descriptor of a conv input
struct LnIn {
    const float* stats = nullptr;
    const float* gamma = nullptr;
    const float* beta = nullptr;
    int act = 0;
};

// debug option TRAIN_ALT bit 32: zero dt1's gradient buffer before the grouped branches' data gradients
// instead of masking the channels outside their windows in the LN2 backward
bool ln2_mask() { return (opts().train_alt & 32) == 0; }

// the LN backward's reduction in the producing data-gradient kernel (TRAIN_ALT bit 16: k_lnb_reduce)
bool fused_lnr() { return (opts().train_alt & 16) == 0; }

int wgrad_chunks(int B, int npx) {
    const long long total = (long long)B * npx;
    return (int)std::max<long long>(1, std::min<long long>(64, (total + 511) / 512));
}

}  // namespace

// LDS pixel stride for C channels: a multiple of 4 floats (16-byte quads), odd in quads
static int bwd_stride(int C) {
    int s = (C + 3) / 4 * 4;
    if (s % 8 == 0) s += 4;
    return s;
}

size_t ldsbwd_setup(const Plan& p, const Coupling& c, LdsBwdArgs& a) {
    std::memset(&a, 0, sizeof(a));
    if (!c.use_lds || (int)c.br.size() > NETLDS_MAXBR || c.bwd_offs_per_net == 0) return 0;
    const int ks = p.desc.ksize, taps = ks * ks;
    if (taps != 1 && taps != 9) return 0;
    for (const Branch& b : c.br)
        if (b.dil > 32) return 0;
    a.H = c.H;
    a.W = c.W;
    a.D = c.D;
    a.mask = c.mask;
    a.hc = c.hc;
    a.wc = c.wc;
    a.dc1 = c.dc1;
    a.dc2 = c.dc2;
    a.nk = c.nk;
    a.gc = c.gc;
    a.R = c.R;
    a.nbr = (int)c.br.size();
    a.ln = p.desc.layer_norm;
    a.taps = taps;
    for (int i = 0; i < a.nbr; i++) {
        a.br_cin_off[i] = c.br[i].cin_off;
        a.br_cin[i] = c.br[i].cin;
        a.br_cout[i] = c.br[i].cout;
        a.br_out_off[i] = c.br[i].out_off;
        a.br_dil[i] = c.br[i].dil;
    }
    const int HW = c.hc * c.wc;
    const int ac = std::max(std::max(c.nk, c.dc1), 4);
    a.sy = bwd_stride(c.nk);
    a.st = bwd_stride(std::max(std::max(c.gc, c.nk), std::max(c.dc2, c.dc1)));
    a.sa = bwd_stride(ac);
    a.ac_chunk = std::min(c.gc, ac / 4 * 4);
    auto kp4 = [](int K) { return (K + 3) / 4 * 4; };
    auto np16 = [](int N) { return (N + 15) / 16 * 16; };
    // transposed-weight images of the data gradients (rows: taps x the output channels rounded up to 4,
    // stage_wt), the k-table lengths of the weight gradients, the zero row of gemm_tap (the widest A)
    size_t wmax = (size_t)taps * kp4(c.dc2) * np16(c.nk);
    wmax = std::max(wmax, (size_t)kp4(c.nk) * np16(c.gc));
    wmax = std::max(wmax, (size_t)kp4(c.nk) * np16(c.nk));
    wmax = std::max(wmax, (size_t)taps * kp4(c.nk) * np16(c.dc1));
    int ktmax = std::max(kp4(taps * c.nk), kp4(taps * c.dc1));
    ktmax = std::max(ktmax, std::max(kp4(c.nk), kp4(a.ac_chunk)));
    int zn = std::max(kp4(c.dc2), kp4(c.nk));
    for (const Branch& b : c.br) {
        wmax = std::max(wmax, (size_t)taps * kp4(b.cout) * np16(b.cin));
        ktmax = std::max(ktmax, kp4(taps * b.cin));
        zn = std::max(zn, kp4(b.cout));
    }
    auto al = [](size_t v) { return (v + 15) / 16 * 16; };
    size_t off = al((size_t)HW * a.sy * 4);
    a.off_gt = (int)off;
    off = al(off + (size_t)HW * a.st * 4);
    a.off_ac = (int)off;
    off = al(off + (size_t)HW * a.sa * 4);
    a.off_w = (int)off;
    a.wmax = (int)wmax;
    off = al(off + wmax * 4);
    a.off_kt = (int)off;
    off = al(off + (size_t)ktmax * 4);
    a.off_red = (int)off;
    off = al(off + 16 * 8);
    a.off_ot = (int)off;
    off = al(off + (size_t)c.bwd_offs_per_net * 4);
    a.off_z = (int)off;   // 4 zeros + 4 ones, then zn + 4 zeros (a lane reads up to kq + cpt4 - 1)
    off = al(off + 32 + (size_t)(zn + 4) * 4);
    if (off > 160 * 1024) return 0;
    a.lds_bytes = (int)off;
    a.offs_per_net = c.bwd_offs_per_net;
    const LdsSave s = LdsSave::of(HW, c.nk, c.gc, c.R);
    a.save_img = s.img;
    a.save_t1 = s.t1;
    a.save_t2 = s.t2;
    a.save_st = s.st;
    a.row = (int)std::max(c.net[0].hi - c.net[0].lo, c.net[1].hi - c.net[1].lo);
    a.gs_rb = HW * (2 * c.nk + c.gc);
    a.g_t3 = HW * c.nk;
    a.g_t2 = HW * (c.nk + c.gc);
    a.g_in = c.R * a.gs_rb;
    a.gsave_img = (a.g_in + HW * c.nk + 3) / 4 * 4;
    return off;
}

TrainLayout Plan::train_layout(int B) const {
    TrainLayout T;
    const WsLayout L = layout(B);
    size_t off = align_up(L.total, 256);
    auto take = [&](size_t bytes) {
        size_t o = off;
        off = align_up(off + std::max<size_t>(bytes, 4), 256);
        return o;
    };
    const size_t Bz = (size_t)B;
    int64_t m_y = 0, m_t1 = 0, m_t2 = 0, m_so = 0, m_nk = 0, m_gc = 0, m_u1 = 0, m_dense = 0, m_co = 0;
    int m_st = 1;
    for (const Coupling& c : couplings) {
        const int64_t npx = (int64_t)c.hc * c.wc;
        m_y = std::max<int64_t>(m_y, (int64_t)(c.R + 1) * npx * c.nk);
        m_t1 = std::max<int64_t>(m_t1, (int64_t)c.R * npx * c.nk);
        m_t2 = std::max<int64_t>(m_t2, (int64_t)c.R * npx * c.gc);
        m_so = std::max<int64_t>(m_so, npx * c.dc2);
        m_nk = std::max<int64_t>(m_nk, npx * c.nk);
        m_gc = std::max<int64_t>(m_gc, npx * c.gc);
        m_u1 = std::max<int64_t>(m_u1, npx * c.dc1);
        m_st = std::max(m_st, 3 * c.R + 1);
        m_dense = std::max<int64_t>(m_dense, 9LL * c.dc1 * c.nk);
        m_dense = std::max<int64_t>(m_dense, (int64_t)c.nk * c.nk);
        m_dense = std::max<int64_t>(m_dense, (int64_t)c.gc * c.nk);
        m_dense = std::max<int64_t>(m_dense, 9LL * c.nk * c.dc2);
        for (const Branch& b : c.br) m_dense = std::max<int64_t>(m_dense, 9LL * b.cin * b.cout);
        m_co = std::max<int64_t>(m_co, std::max(std::max(c.nk, c.dc2), c.gc));
    }
    T.save_u.assign(couplings.size(), 0);
    for (const Coupling& c : couplings) T.save_u[c.index] = take(Bz * c.H * c.W * c.D * 4);
    T.bw = take((size_t)std::max<int64_t>(n_bw, 1) * 4);
    for (int n = 0; n < 2; n++) {
        T.ys[n] = take(Bz * m_y * 4);
        T.t1s[n] = take(Bz * m_t1 * 4);
        T.t2s[n] = take(Bz * m_t2 * 4);
        T.so[n] = take(Bz * m_so * 4);
        T.dso[n] = take(Bz * m_so * 4);
        T.stats[n] = take(Bz * m_st * 2 * 4);
    }
    for (int n = 0; n < 2; n++) {
        T.dy[n] = take(Bz * m_nk * 4);
        T.dln[n] = take(Bz * m_nk * 4);
        T.dbuf[n] = take(Bz * m_nk * 4);
        T.dt1[n] = take(Bz * m_nk * 4);
        T.dc[n] = take(Bz * m_gc * 4);
        T.dt2[n] = take(Bz * m_gc * 4);
        T.du1c[n] = take(Bz * m_u1 * 4);
    }
    T.u1c = take(Bz * m_u1 * 4);
    for (int k = 0; k < 2; k++) T.duv[k] = take(Bz * L.n_uv * 4);
    T.dzy = take(Bz * L.n_uv * 4);
    for (int n = 0; n < 2; n++) {
        T.lnsum[n] = take(Bz * std::max(LNB_RS, LNR_MAXPARTS) * 2 * 8);
        // LN backward: per batch slice partial gamma / beta gradients [2][LNB_SLICES][n]
        T.lnpart[n] = take((size_t)2 * LNB_SLICES * std::max(m_nk, m_gc) * 4);
    }
    int chunks = 1, mchunks = WGRAD_MAX_CHUNKS;
    for (const Coupling& c : couplings) {
        chunks = std::max(chunks, wgrad_chunks(B, c.hc * c.wc));
        mchunks = std::max(mchunks, wgrad_direct_chunks(B, c.hc));   // (B of them once B > WGRAD_MAX_CHUNKS)
    }
    // the MFMA weight gradients write up to mchunks rows of [weights | bias]
    for (int n = 0; n < 2; n++) {
        T.wpart[n] = take((size_t)std::max(chunks, mchunks) * (m_dense + m_co) * 4);
        T.bpart[n] = take((size_t)chunks * m_co * 4);
    }
    T.dwpart = take(Bz * std::max(1, L.ld_parts) * 8);
    T.zeros = take(64 * 4);
    T.act_save.assign(couplings.size(), 0);
    T.so_save.assign(couplings.size(), 0);
    for (const Coupling& c : couplings) {
        if (!c.lds_bwd) continue;
        const int HW = c.hc * c.wc;
        const LdsSave s = LdsSave::of(HW, c.nk, c.gc, c.R);
        T.act_save[c.index] = take(2 * Bz * s.img * 4);
        T.so_save[c.index] = take(2 * Bz * HW * c.dc2 * 4);
        T.row_max = std::max<int>(T.row_max, (int)std::max(c.net[0].hi - c.net[0].lo, c.net[1].hi - c.net[1].lo));
    }
    if (T.row_max > 0) {
        T.rows = take(2 * Bz * T.row_max * 4);
        T.rows2 = take(2 * Bz * T.row_max * 4);
        for (const Coupling& c : couplings) {
            if (!c.lds_bwd) continue;
            const int HW = c.hc * c.wc;
            T.gsave_max = std::max(T.gsave_max, ((c.R * (2 * c.nk + c.gc) + c.nk) * HW + 3) / 4 * 4);
        }
        for (int par = 0; par < 2; par++) {
            T.gsave[par] = take(2 * Bz * T.gsave_max * 4);
            for (int n = 0; n < 2; n++) T.dso_l[par][n] = take(Bz * m_so * 4);
        }
    }
    // streamed layers' saved activations, when all of them fit 16 GiB (TRAIN_SCHED bit 2: recompute)
    T.ssave.assign(couplings.size(), TrainLayout::StreamSave{});
    T.has_ssave.assign(couplings.size(), 0);
    {
        const bool on = (opts.train_sched & 2) == 0;
        size_t need = 0;
        for (const Coupling& c : couplings) {
            if (c.use_lds || c.t2_mapped) continue;
            const size_t npx = (size_t)c.hc * c.wc;
            need += 2 * Bz * npx * ((size_t)(c.R + 1) * c.nk + (size_t)c.R * c.nk + (size_t)c.R * c.gc + c.dc2) * 4;
        }
        if (on && need <= (16ull << 30))
            for (const Coupling& c : couplings) {
                if (c.use_lds || c.t2_mapped) continue;
                const size_t npx = (size_t)c.hc * c.wc;
                TrainLayout::StreamSave& s = T.ssave[c.index];
                for (int n = 0; n < 2; n++) {
                    s.y[n] = take((size_t)(c.R + 1) * Bz * npx * c.nk * 4);
                    s.t1[n] = take((size_t)std::max(c.R, 1) * Bz * npx * c.nk * 4);
                    s.t2[n] = take((size_t)std::max(c.R, 1) * Bz * npx * c.gc * 4);
                    s.st[n] = take((size_t)(3 * c.R + 1) * Bz * 2 * 4);
                }
                s.so = take(2 * Bz * npx * c.dc2 * 4);
                T.has_ssave[c.index] = 1;
            }
    }
    T.total = off;
    return T;
}

namespace {

struct TExec {
    Plan& p;
    const float* params;
    float* dparams;
    char* ws;
    WsLayout L;
    TrainLayout T;
    int B;
    hipStream_t st;
    float inv_batch_ = 0.f;
    const float* count = nullptr;   // device global image count (overrides inv_batch_)
    bool saved = false;             // the training forward saved the streamed layers' activations (flow backward)
    int net = 0;   // which per-net scratch set (and stream) this executor's launches use
    hipStream_t wst = nullptr;   // weight-gradient stream (null: on st)
    const float* bw() const { return reinterpret_cast<const float*>(ws + T.bw); }
    template <class X>
    X* at(size_t off) const {
        return reinterpret_cast<X*>(ws + off);
    }
};

// out = conv(in) over the dense image of pc (forward, sgn = +1)
void conv_fwd(TExec& E, int h, int w, const float* in, int in_cs, int in_off, int K, const LnIn& ln,
              const PackedConv& pc, int cout, int dil, const float* res, float* out, int out_cs, int out_off) {
    TConvArgs a{};
    a.in = in;
    a.in_cs = in_cs;
    a.in_off = in_off;
    a.K = K;
    a.stats = ln.stats;
    a.gamma = ln.gamma;
    a.beta = ln.beta;
    a.act = ln.act;
    a.w = E.bw() + pc.dw;
    a.wt = (long long)K * cout;
    a.wk = cout;
    a.wn = 1;
    a.bias = E.bw() + pc.db;
    a.res = res;
    a.out = out;
    a.out_cs = out_cs;
    a.out_off = out_off;
    a.N = cout;
    a.accumulate = 0;
    a.H = h;
    a.W = w;
    a.taps = pc.taps;
    a.dil = dil;
    a.sgn = 1;
    a.B = E.B;
    a.zero = E.at<float>(E.T.zeros);
    launch_tconv(a, E.st);
}

// dx (=|+=) conv^T(dy): dy has cout channels at (dy_cs, dy_off), dx gets cin channels at (dx_cs, dx_off)
// With lr (an LN whose input has dx's layout and whose output gradient dx is), the kernel also writes the
// LN backward's per-image reduction partials to the net's lnsum; returns their count per image (0: not
// fused — ln_bwd runs k_lnb_reduce)
struct LnRed {
    const float* x = nullptr;
    const float* gamma = nullptr;
    const float* stats = nullptr;
    int base = 0;   // this launch's first partial (several launches that write disjoint windows share one LN)
};
int conv_dgrad(TExec& E, int h, int w, const float* dy, int dy_cs, int dy_off, int cout, const PackedConv& pc, int cin,
               int dil, float* dx, int dx_cs, int dx_off, int accumulate, const LnRed* lr = nullptr) {
    TConvArgs a{};
    if (lr != nullptr && lr->stats != nullptr && fused_lnr()) {
        a.lnr_x = lr->x;
        a.lnr_gamma = lr->gamma;
        a.lnr_stats = lr->stats;
        a.lnr_part = E.at<double>(E.T.lnsum[E.net]);
        a.lnr_base = lr->base;
        a.lnr_stride = LNR_MAXPARTS;
    }
    a.in = dy;
    a.in_cs = dy_cs;
    a.in_off = dy_off;
    a.K = cout;
    a.w = E.bw() + pc.dw;
    a.wt = (long long)cin * cout;
    a.wk = 1;
    a.wn = cout;
    a.out = dx;
    a.out_cs = dx_cs;
    a.out_off = dx_off;
    a.N = cin;
    a.accumulate = accumulate;
    a.H = h;
    a.W = w;
    a.taps = pc.taps;
    a.dil = dil;
    a.sgn = -1;
    a.B = E.B;
    a.zero = E.at<float>(E.T.zeros);
    return launch_tconv(a, E.st);
}

// dW, db of a conv: X (cin channels at x_cs/x_off, LN-on-load) and dY (cout at dy_cs/dy_off)
hipEvent_t tevent(Plan& p) {
    constexpr int flags = (int)hipEventDisableTiming;
    if (p.tev_next == p.tev.size()) {
        hipEvent_t e;
        hchk(hipEventCreateWithFlags(&e, flags), "hipEventCreate");
        p.tev.push_back(e);
    }
    return p.tev[p.tev_next++];
}

// dW, db of a conv (below) on E's weight-gradient stream when it has one: it waits for the chain's
// launches so far (its X and dY are ready) and returns the event of its completion, which the chain
// waits for before it overwrites that dY buffer
hipEvent_t conv_wgrad_impl(TExec& E, int h, int w, const float* x, int x_cs, int x_off, int cin, const LnIn& ln,
                           const float* dy, int dy_cs, int dy_off, int cout, const PackedConv& pc, int dil);
hipEvent_t conv_wgrad(TExec& E, int h, int w, const float* x, int x_cs, int x_off, int cin, const LnIn& ln,
                      const float* dy, int dy_cs, int dy_off, int cout, const PackedConv& pc, int dil) {
    if (E.wst == nullptr) {
        conv_wgrad_impl(E, h, w, x, x_cs, x_off, cin, ln, dy, dy_cs, dy_off, cout, pc, dil);
        return nullptr;
    }
    hipEvent_t in = tevent(E.p), done = tevent(E.p);
    hchk(hipEventRecord(in, E.st), "hipEventRecord");
    hchk(hipStreamWaitEvent(E.wst, in, 0), "hipStreamWaitEvent");
    TExec G = E;
    G.st = E.wst;
    conv_wgrad_impl(G, h, w, x, x_cs, x_off, cin, ln, dy, dy_cs, dy_off, cout, pc, dil);
    hchk(hipEventRecord(done, E.wst), "hipEventRecord");
    return done;
}

void chain_wait(TExec& E, hipEvent_t done) {
    if (done != nullptr) hchk(hipStreamWaitEvent(E.st, done, 0), "hipStreamWaitEvent");
}

hipEvent_t conv_wgrad_impl(TExec& E, int h, int w, const float* x, int x_cs, int x_off, int cin, const LnIn& ln,
                           const float* dy, int dy_cs, int dy_off, int cout, const PackedConv& pc, int dil) {
    WGradArgs a{};
    a.x = x;
    a.x_cs = x_cs;
    a.x_off = x_off;
    a.CI = cin;
    a.stats = ln.stats;
    a.gamma = ln.gamma;
    a.beta = ln.beta;
    a.act = ln.act;
    a.dy = dy;
    a.dy_cs = dy_cs;
    a.dy_off = dy_off;
    a.CO = cout;
    a.part = E.at<float>(E.T.wpart[E.net]);
    a.bpart = E.at<float>(E.T.bpart[E.net]);
    a.H = h;
    a.W = w;
    a.taps = pc.taps;
    a.dil = dil;
    a.B = E.B;
    const int64_t* map = E.p.dev_bw_map;
    const long long nw = (long long)pc.taps * cin * cout;
    if (train_valu_kernels() || !wgrad_band_ok(h, w, pc.taps, dil, cin, cout)) {
        a.chunks = wgrad_chunks(E.B, h * w);
        const long long total = (long long)E.B * h * w;
        a.chunk_px = (int)(((total + a.chunks - 1) / a.chunks + 15) / 16 * 16);
        launch_wgrad(a, E.st);
        launch_grad_scatter(a.part, a.chunks, nw, map + pc.dw, E.dparams, E.st);
        launch_grad_scatter(a.bpart, a.chunks, cout, map + pc.db, E.dparams, E.st);
        return nullptr;
    }
    // thin outputs (the streamed conv_out, CO = dc2): k_wgrad_thin, rows of [weights | bias] as below
    if ((long long)h * w * x_cs * 4 < (1LL << 31) && wgrad_thin_ok(h, w, pc.taps, dil, cin, cout) && pc.db == pc.dw + nw) {
        a.chunks = wgrad_thin_chunks(E.B, h, w);
        launch_wgrad_thin(a, E.st);
        launch_grad_scatter(a.part, a.chunks, nw + cout, map + pc.dw, E.dparams, E.st);
        return nullptr;
    }
    // k_wgrad_direct (k_wgrad_band with TRAIN_ALT bit 2): rows of [weights | bias]; the dense image
    // keeps the bias right after the weights (pc.db == pc.dw + taps * cin * cout), so one scatter
    // reduces both
    const bool direct = (opts().train_alt & 2) == 0;
    if (direct && wgrad_direct_ok(h, w, pc.taps)) {
        a.chunks = wgrad_direct_chunks(E.B, h);
        a.chunk_px = -1;
        a.zero = E.at<float>(E.T.zeros);
    } else {
        a.chunks = wgrad_band_chunks(E.B, h, w, pc.taps, cin, cout);
    }
    launch_wgrad(a, E.st);
    if (pc.db != pc.dw + nw) throw std::logic_error("dense image: bias not after the weights");
    launch_grad_scatter(a.part, a.chunks, nw + cout, map + pc.dw, E.dparams, E.st);
    return nullptr;
}

void ln_bwd(TExec& E, const float* x, const float* dxo, const LnIn& ln, long long n, float* dx, int accumulate,
            int64_t g_off, int64_t b_off, int presum = 0, unsigned long long cmask = 0, int cmod = 0) {
    launch_ln_backward(x, dxo, ln.gamma, ln.stats, E.at<double>(E.T.lnsum[E.net]), n, E.B, 1, dx, accumulate,
                       ln.stats ? E.dparams + g_off : nullptr, ln.stats ? E.dparams + b_off : nullptr,
                       E.at<float>(E.T.lnpart[E.net]), E.st, presum, LNR_MAXPARTS, cmask, cmod);
}

// the plan's side stream and fork / join events (created on first use on the current device)
void ensure_side(Plan& p) {
    int dev = 0;
    hchk(hipGetDevice(&dev), "hipGetDevice");
    if (p.side != nullptr && p.side_device == dev) return;
    if (p.side != nullptr) {
        (void)hipEventDestroy(p.ev_fork);
        (void)hipEventDestroy(p.ev_join);
        (void)hipStreamDestroy(p.side);
        for (hipStream_t& s : p.wside) (void)hipStreamDestroy(s);
        p.side = nullptr;
        // the pooled events belong to the old device too: recording them on the new device's streams fails
        for (hipEvent_t e : p.tev) (void)hipEventDestroy(e);
        p.tev.clear();
        p.tev_next = 0;
    }
    hchk(hipStreamCreateWithFlags(&p.side, hipStreamNonBlocking), "hipStreamCreate");
    hchk(hipEventCreateWithFlags(&p.ev_fork, hipEventDisableTiming), "hipEventCreate");
    hchk(hipEventCreateWithFlags(&p.ev_join, hipEventDisableTiming), "hipEventCreate");
    for (hipStream_t& s : p.wside) hchk(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    p.side_device = dev;
}

// `to` waits for everything enqueued on `from` so far
void stream_wait(hipStream_t from, hipStream_t to, hipEvent_t ev) {
    hchk(hipEventRecord(ev, from), "hipEventRecord");
    hchk(hipStreamWaitEvent(to, ev, 0), "hipStreamWaitEvent");
}

// One coupling layer's backward (conv_cINN_make_model.py:1850-1880 through the layer): the two s,t
// nets are independent until the coupling law joins them, so net b's recompute and backward chain run
// on the plan's side stream (its own scratch set) while net A's run on the caller's stream: the many
// small, latency-bound launches of the two chains overlap.
// the fused backward of a k_net_lds layer (cnf_ldsbwd.hip) from the activations the training forward
// saved: coupling law backward, one k_lds_bwd launch for both nets, the batch sum of the gradient rows
// the fused backward of a k_net_lds layer (cnf_ldsbwd.hip) from the activations the training forward
// saved: coupling law backward, k_lds_bwd for both nets, the batch sum of the gradient rows. Split
// (par >= 0): the data-gradient chain (k_lds_bwd mode 1, storing the gradients the weight gradients
// need) on the caller's stream, then the weight gradients (mode 2) and the row sum on the side stream
// wside[1] behind an event, so they run on the CUs the next layer's chain leaves idle (one workgroup per
// (image, net) fills half the GPU at B = 64); returns the event of the row sum (the layer's parameter
// gradients complete), null unsplit. par selects the alternating buffer set.
hipEvent_t coupling_backward_lds(TExec& E, const Coupling& c, const float* u, const float* dv, float* du, int par) {
    const int B = E.B;
    const float* P = E.params;
    const bool split = par >= 0;
    const float* so0 = E.at<float>(E.T.so_save[c.index]);
    float* dso0 = E.at<float>(split ? E.T.dso_l[par][0] : E.T.dso[0]);
    float* dso1 = E.at<float>(split ? E.T.dso_l[par][1] : E.T.dso[1]);
    {
        CoupBwArgs a{};
        a.u = u;
        a.dv = dv;
        a.s_pre = so0;
        a.tanh_w = P + c.net[0].tanh_w;
        a.du = du;
        a.ds_pre = dso0;
        a.dt = dso1;
        a.dw_part = E.at<double>(E.T.dwpart);
        a.g_ld = -E.inv_batch_;
        a.count = E.count;
        a.H = c.H;
        a.W = c.W;
        a.D = c.D;
        a.mask = c.mask;
        a.mask_c = c.mask_c;
        a.hc = c.hc;
        a.wc = c.wc;
        a.dc1 = c.dc1;
        a.dc2 = c.dc2;
        const int np = std::max(1, E.L.ld_parts);
        launch_coupling_backward(a, B, np, E.st);
        launch_dsum(a.dw_part, (long long)B * np, E.dparams + c.net[0].tanh_w, E.st);
    }
    LdsBwdArgs a;
    if (ldsbwd_setup(E.p, c, a) == 0) throw std::logic_error("fused LDS backward planned for a layer it does not fit");
    a.save = E.at<float>(E.T.act_save[c.index]);
    a.dso[0] = dso0;
    a.dso[1] = dso1;
    a.u = u;
    a.du1c[0] = E.at<float>(E.T.du1c[0]);
    a.du1c[1] = E.at<float>(E.T.du1c[1]);
    a.params = P;
    a.bw = E.bw();
    a.bw_map = E.p.dev_bw_map;
    a.offs = E.p.dev_table + c.dev_bwd_offs;
    a.part = E.at<float>(split && par == 1 ? E.T.rows2 : E.T.rows);
    a.row = E.T.row_max;
#ifdef CNF_DIAG
    static const bool stamps = [] {   // diagnostic builds: phase stamps (profiles/diag/diag_bwd_stamps.py)
        const char* e = std::getenv("CNF_LDSBWD_STAMPS");
        return e && std::atoi(e) != 0;
    }();
#else
    constexpr bool stamps = false;
#endif
    a.stamps = stamps ? 1 : 0;
    const NetParams& n0 = c.net[0];
    const NetParams& n1 = c.net[1];
    if (!split) {
        a.mode = 0;
        launch_lds_bwd(a, B, E.st);
        launch_grad_rows(a.part, B, a.row, n0.lo, n1.lo, (int)(n0.hi - n0.lo), (int)(n1.hi - n1.lo), E.dparams, E.st);
        launch_scatter_add_u1c(a.du1c[0], du, B, c.H, c.W, c.D, c.mask, c.hc, c.wc, c.dc1, E.st);
        launch_scatter_add_u1c(a.du1c[1], du, B, c.H, c.W, c.D, c.mask, c.hc, c.wc, c.dc1, E.st);
        return nullptr;
    }
    ensure_side(E.p);
    a.gsave = E.at<float>(E.T.gsave[par]);
    a.mode = 1;
    launch_lds_bwd(a, B, E.st);
    launch_scatter_add_u1c(a.du1c[0], du, B, c.H, c.W, c.D, c.mask, c.hc, c.wc, c.dc1, E.st);
    launch_scatter_add_u1c(a.du1c[1], du, B, c.H, c.W, c.D, c.mask, c.hc, c.wc, c.dc1, E.st);
    hipStream_t ws = E.p.wside[1];
    stream_wait(E.st, ws, tevent(E.p));   // the chain's stored gradients and LN rows
    a.mode = 2;
    a.stamps = 0;
    launch_lds_bwd(a, B, ws);
    launch_grad_rows(a.part, B, a.row, n0.lo, n1.lo, (int)(n0.hi - n0.lo), (int)(n1.hi - n1.lo), E.dparams, ws);
    hipEvent_t done = tevent(E.p);
    hchk(hipEventRecord(done, ws), "hipEventRecord");
    return done;
}

void coupling_backward(TExec& E, const Coupling& c, const float* u, const float* dv, float* du) {
    const int B = E.B, h = c.hc, w = c.wc, nk = c.nk, gc = c.gc, R = c.R;
    const int64_t npx = (int64_t)h * w;
    const bool ln = E.p.desc.layer_norm != 0;
    const float* P = E.params;
    ensure_side(E.p);
    const bool wstreams = (opts().train_sched & 1) == 0;   // TRAIN_SCHED bit 1: weight gradients on the chain streams
    TExec E0 = E;
    E0.wst = wstreams ? E.p.wside[0] : nullptr;
    TExec E1 = E;
    E1.net = 1;
    E1.st = E.p.side;
    E1.wst = wstreams ? E.p.wside[1] : nullptr;
    TExec* X[2] = {&E0, &E1};
    float* u1c = E.at<float>(E.T.u1c);
    launch_gather_u1c(u, u1c, B, c.H, c.W, c.D, c.mask, h, w, c.dc1, E.st);
    // activations of both nets: y_r (r = 0..R), t1_r, t2_r; LN stats st[0..R] (y), st[R+1+r] (t1),
    // st[2R+1+r] (t2), each [B][2]
    // the training forward's saved activations of this (streamed) layer, when it saved them (the backward
    // of a lone layer, cnf_coupling_backward, always recomputes)
    const bool saved = E.saved && E.T.has_ssave[c.index];
    const TrainLayout::StreamSave& SS = E.T.ssave[c.index];
    auto Y = [&](int n, int r) { return E.at<float>(saved ? SS.y[n] : E.T.ys[n]) + (size_t)r * B * npx * nk; };
    auto T1 = [&](int n, int r) { return E.at<float>(saved ? SS.t1[n] : E.T.t1s[n]) + (size_t)r * B * npx * nk; };
    auto T2 = [&](int n, int r) { return E.at<float>(saved ? SS.t2[n] : E.T.t2s[n]) + (size_t)r * B * npx * gc; };
    auto ST = [&](int n, int i) { return E.at<float>(saved ? SS.st[n] : E.T.stats[n]) + (size_t)i * B * 2; };
    auto SO = [&](int n) { return saved ? E.at<float>(SS.so) + (size_t)n * B * npx * c.dc2 : E.at<float>(E.T.so[n]); };
    auto lnin = [&](int n, int i, int64_t g, int64_t b) {
        LnIn l;
        l.act = 1;
        if (ln) {
            l.stats = ST(n, i);
            l.gamma = P + g;
            l.beta = P + b;
        }
        return l;
    };
    const LnIn raw{};
    stream_wait(E.st, E1.st, tevent(E.p));   // u1c gathered
    for (int n = 0; n < 2 && !saved; n++) {
        TExec& En = *X[n];
        const NetParams& np = c.net[n];
        conv_fwd(En, h, w, u1c, c.dc1, 0, c.dc1, raw, np.ci, nk, 1, nullptr, Y(n, 0), nk, 0);
        if (ln) launch_ln_stats(Y(n, 0), npx * nk, B, 1, ST(n, 0), En.st);
        for (int r = 0; r < R; r++) {
            const RBParams& rb = np.rb[r];
            conv_fwd(En, h, w, Y(n, r), nk, 0, nk, lnin(n, r, rb.ln1g, rb.ln1b), rb.ca, nk, 1, nullptr, T1(n, r), nk, 0);
            if (ln) launch_ln_stats(T1(n, r), npx * nk, B, 1, ST(n, R + 1 + r), En.st);
            for (size_t bi = 0; bi < c.br.size(); bi++) {
                const Branch& b = c.br[bi];
                conv_fwd(En, h, w, T1(n, r), nk, b.cin_off, b.cin, lnin(n, R + 1 + r, rb.ln2g, rb.ln2b), rb.gc[bi],
                         b.cout, b.dil, nullptr, T2(n, r), gc, b.out_off);
            }
            if (ln) launch_ln_stats(T2(n, r), npx * gc, B, 1, ST(n, 2 * R + 1 + r), En.st);
            conv_fwd(En, h, w, T2(n, r), gc, 0, gc, lnin(n, 2 * R + 1 + r, rb.ln3g, rb.ln3b), rb.cb, nk, 1, Y(n, r),
                     Y(n, r + 1), nk, 0);
            if (ln) launch_ln_stats(Y(n, r + 1), npx * nk, B, 1, ST(n, r + 1), En.st);
        }
        conv_fwd(En, h, w, Y(n, R), nk, 0, nk, lnin(n, R, np.ln_out_g, np.ln_out_b), np.co, c.dc2, 1, nullptr,
                 SO(n), c.dc2, 0);
    }
    stream_wait(E1.st, E.st, tevent(E.p));   // both nets' outputs
    // coupling law backward -> du (u2 part, u1 copy), dL/d s_pre, dL/dt, dL/dw
    {
        CoupBwArgs a{};
        a.u = u;
        a.dv = dv;
        a.s_pre = SO(0);
        a.tanh_w = P + c.net[0].tanh_w;
        a.du = du;
        a.ds_pre = E.at<float>(E.T.dso[0]);
        a.dt = E.at<float>(E.T.dso[1]);
        a.dw_part = E.at<double>(E.T.dwpart);
        a.g_ld = -E.inv_batch_;
        a.count = E.count;
        a.H = c.H;
        a.W = c.W;
        a.D = c.D;
        a.mask = c.mask;
        a.mask_c = c.mask_c;
        a.hc = h;
        a.wc = w;
        a.dc1 = c.dc1;
        a.dc2 = c.dc2;
        const int np = std::max(1, E.L.ld_parts);
        launch_coupling_backward(a, B, np, E.st);
        launch_dsum(a.dw_part, (long long)B * np, E.dparams + c.net[0].tanh_w, E.st);
    }
    stream_wait(E.st, E1.st, tevent(E.p));   // dL/d s_pre, dL/dt
    // The two chains are enqueued interleaved, phase by phase (conv_out; per residual block conv_b + LN3,
    // the branches + LN2, conv_a + LN1; conv_in): the GPU starts a stream's kernels in about the order
    // the host submitted them across streams (measured: no kernel ran more than ~15 submissions ahead of
    // the newest finished one), so a chain enqueued whole after the other only overlapped it at the end.
    // Debug option TRAIN_SCHED bit 4 enqueues net A's chain, then net b's.
    const bool interleave = (opts().train_sched & 4) == 0;
    hipEvent_t ev_gc[2] = {nullptr, nullptr}, ev_ca[2] = {nullptr, nullptr}, ev_cb[2] = {nullptr, nullptr};
    // phase k of net n: 0 conv_out + LN_out; 1 + 3j + {0, 1, 2} residual block r = R - 1 - j: conv_b + LN3,
    // the grouped branches + LN2, conv_a + LN1; 1 + 3R conv_in
    auto phase = [&](int n, int k) {
        TExec& En = *X[n];
        float* dy = E.at<float>(E.T.dy[n]);
        float* dln = E.at<float>(E.T.dln[n]);
        float* dbuf = E.at<float>(E.T.dbuf[n]);
        float* dt1 = E.at<float>(E.T.dt1[n]);
        float* dcb = E.at<float>(E.T.dc[n]);
        float* dt2 = E.at<float>(E.T.dt2[n]);
        float* du1c = E.at<float>(E.T.du1c[n]);
        const NetParams& np = c.net[n];
        if (k == 0) {
            const float* dso = E.at<float>(E.T.dso[n]);
            const LnIn lo = lnin(n, R, np.ln_out_g, np.ln_out_b);
            conv_wgrad(En, h, w, Y(n, R), nk, 0, nk, lo, dso, c.dc2, 0, c.dc2, np.co, 1);
            const LnRed ro{Y(n, R), lo.gamma, lo.stats};
            const int ps = conv_dgrad(En, h, w, dso, c.dc2, 0, c.dc2, np.co, nk, 1, dln, nk, 0, 0, &ro);
            ln_bwd(En, Y(n, R), dln, lo, npx * nk, dy, 0, np.ln_out_g, np.ln_out_b, ps);
            return;
        }
        if (k == 1 + 3 * R) {
            conv_wgrad(En, h, w, u1c, c.dc1, 0, c.dc1, raw, dy, nk, 0, nk, np.ci, 1);
            conv_dgrad(En, h, w, dy, nk, 0, nk, np.ci, c.dc1, 1, du1c, c.dc1, 0, 0);
            return;
        }
        // the weight gradients run behind the chain on En.wst; before the chain overwrites a dY buffer
        // it waits for the weight gradients reading it (of the block before: dt2, dt1; this block: dy)
        const int r = R - 1 - (k - 1) / 3, part = (k - 1) % 3;
        const RBParams& rb = np.rb[r];
        if (part == 0) {   // conv_b (y_{r+1} = y_r + conv_b(LN3(t2_r)))
            const LnIn l3 = lnin(n, 2 * R + 1 + r, rb.ln3g, rb.ln3b);
            ev_cb[n] = conv_wgrad(En, h, w, T2(n, r), gc, 0, gc, l3, dy, nk, 0, nk, rb.cb, 1);
            const LnRed r3{T2(n, r), l3.gamma, l3.stats};
            const int ps = conv_dgrad(En, h, w, dy, nk, 0, nk, rb.cb, gc, 1, dcb, gc, 0, 0, &r3);
            chain_wait(En, ev_gc[n]);
            ln_bwd(En, T2(n, r), dcb, l3, npx * gc, dt2, 0, rb.ln3g, rb.ln3b, ps);
        } else if (part == 1) {   // grouped dilated branches
            const LnIn l2 = lnin(n, R + 1 + r, rb.ln2g, rb.ln2b);
            // the LN2 reduction rides on the branches' data gradients when their windows are pairwise disjoint
            // (the reference group mode's closure windows [(card - 1) w, card w) of each branch width w): each
            // element of dbuf is then final after the one launch that writes it, and each launch adds its
            // window's partials after the previous launches'
            const int nb = (int)c.br.size();
            bool disjoint = true;
            unsigned long long wmask = 0;
            for (int i = 0; i < nb; i++) {
                for (int j = i + 1; j < nb; j++)
                    disjoint = disjoint && (c.br[i].cin_off + c.br[i].cin <= c.br[j].cin_off ||
                                            c.br[j].cin_off + c.br[j].cin <= c.br[i].cin_off);
                for (int ch = c.br[i].cin_off; ch < c.br[i].cin_off + c.br[i].cin && ch < 64; ch++) wmask |= 1ull << ch;
            }
            // disjoint windows over <= 64 channels: the branches store their windows (no accumulate) and the
            // LN2 backward reads the channels outside them as 0 (channel mask), so dbuf is not zeroed first
            const bool masked = disjoint && nk <= 64 && ln2_mask();
            if (!masked) hchk(hipMemsetAsync(dbuf, 0, (size_t)B * npx * nk * 4, En.st), "hipMemsetAsync");
            int ps = 0;
            bool fused = disjoint;
            for (int bi = 0; bi < nb; bi++) {
                const Branch& b = c.br[bi];
                ev_gc[n] = conv_wgrad(En, h, w, T1(n, r), nk, b.cin_off, b.cin, l2, dt2, gc, b.out_off, b.cout,
                                      rb.gc[bi], b.dil);
                LnRed r2{T1(n, r), l2.gamma, l2.stats};
                r2.base = ps;
                const int np = conv_dgrad(En, h, w, dt2, gc, b.out_off, b.cout, rb.gc[bi], b.cin, b.dil, dbuf, nk,
                                          b.cin_off, masked ? 0 : 1, fused ? &r2 : nullptr);
                fused = fused && np > 0;
                ps += np;
            }
            if (!fused) ps = 0;   // (k_lnb_reduce, over whatever partials were written)
            chain_wait(En, ev_ca[n]);
            ln_bwd(En, T1(n, r), dbuf, l2, npx * nk, dt1, 0, rb.ln2g, rb.ln2b, ps, masked ? wmask : 0ull,
                   masked ? nk : 0);
        } else {   // conv_a
            const LnIn l1 = lnin(n, r, rb.ln1g, rb.ln1b);
            ev_ca[n] = conv_wgrad(En, h, w, Y(n, r), nk, 0, nk, l1, dt1, nk, 0, nk, rb.ca, 1);
            const LnRed r1{Y(n, r), l1.gamma, l1.stats};
            const int ps = conv_dgrad(En, h, w, dt1, nk, 0, nk, rb.ca, nk, 1, dln, nk, 0, 0, &r1);
            chain_wait(En, ev_cb[n]);
            ln_bwd(En, Y(n, r), dln, l1, npx * nk, dy, 1, rb.ln1g, rb.ln1b, ps);
        }
    };
    const int nphase = 2 + 3 * R;
    if (interleave) {
        for (int k = 0; k < nphase; k++)
            for (int n = 0; n < 2; n++) phase(n, k);
    } else {
        for (int n = 0; n < 2; n++)
            for (int k = 0; k < nphase; k++) phase(n, k);
    }
    stream_wait(E1.st, E.st, tevent(E.p));   // net b's chain done
    for (int n = 0; n < 2; n++)                  // and both nets' weight gradients
        if (X[n]->wst) stream_wait(X[n]->wst, E.st, tevent(E.p));
    // du += the two nets' u1 gradients, net A's first (fixed order: bitwise reproducible)
    launch_scatter_add_u1c(E.at<float>(E.T.du1c[0]), du, B, c.H, c.W, c.D, c.mask, h, w, c.dc1, E.st);
    launch_scatter_add_u1c(E.at<float>(E.T.du1c[1]), du, B, c.H, c.W, c.D, c.mask, h, w, c.dc1, E.st);
}

}  // namespace

void flow_backward(Plan& p, const float* params, const float* xy, const float* zy, void* workspace, int B,
                   float inv_batch, float* dparams, hipStream_t st, const float* count, LayerDoneFn done, void* user) {
    TExec E{p, params, dparams, (char*)workspace, p.layout(B), p.train_layout(B), B, st};
    E.inv_batch_ = inv_batch;
    E.count = count;
    E.saved = true;
    // pooled events: each record of this call gets its own (a re-recorded event that a queued wait still
    // references serialised the two nets' chains on the GPU); the previous call's waits are all enqueued
    p.tev_next = 0;
    const WsLayout& L = E.L;
    const int* T = p.dev_table;
    if (p.n_bw > 0) launch_pack(params, p.dev_bw_map, E.at<float>(E.T.bw), (long long)p.n_bw, st);
    hchk(hipMemsetAsync(dparams, 0, (size_t)p.n_params * 4, st), "hipMemsetAsync");
    hchk(hipMemsetAsync(E.at<float>(E.T.zeros), 0, 64 * 4, st), "hipMemsetAsync");
    const int nuv = (int)L.n_uv;
    const cnf_flow_desc& d = p.desc;
    float* dzy = E.at<float>(E.T.dzy);
    launch_nll_grad(xy, zy, dzy, B, d.io_h * d.io_w, d.io_d, d.x_d, d.lambda_y, inv_batch, count, st);
    float* buf[2] = {E.at<float>(E.T.duv[0]), E.at<float>(E.T.duv[1])};
    int which = 0;
    launch_map_gather(dzy, buf[which], T + p.dev_final_orig, p.last_n, nuv, p.last_n, B, st);
    float* cur = buf[which];
    which ^= 1;
    int bi = (int)p.boundaries.size() - 1;
    // split LDS layers: their weight gradients finish behind the next layers on a side stream; a layer's
    // buffer set (parity of its LDS-layer count) is reused two LDS layers later, when the caller's stream
    // first waits for them — that is also when the layer's gradients are complete for `done`
    const bool split = opts().lds_bwd == 2;   // (debug option LDS_BWD=1: one launch per layer)
    struct Pending {
        int ci = -1;
        hipEvent_t ev = nullptr;
    } pend[2];
    auto flush = [&](int par) {
        if (pend[par].ci < 0) return;
        hchk(hipStreamWaitEvent(st, pend[par].ev, 0), "hipStreamWaitEvent");
        if (done != nullptr) done(user, pend[par].ci);
        pend[par].ci = -1;
    };
    int lds_k = 0;
    for (int li = (int)p.layers.size() - 1; li >= 0; li--) {
        const Layer& ly = p.layers[li];
        if (ly.kind == CNF_LAYER_COUPLING) {
            const Coupling& c = p.couplings[ly.ci];
            float* nxt = buf[which];
            if (c.lds_bwd && split) {
                const int par = lds_k++ & 1;
                flush(par);
                pend[par].ev = coupling_backward_lds(E, c, E.at<float>(E.T.save_u[c.index]), cur, nxt, par);
                pend[par].ci = c.index;
            } else {
                if (c.lds_bwd)
                    coupling_backward_lds(E, c, E.at<float>(E.T.save_u[c.index]), cur, nxt, -1);
                else
                    coupling_backward(E, c, E.at<float>(E.T.save_u[c.index]), cur, nxt);
                // every launch writing this layer's parameter gradients is ordered before anything enqueued
                // on st from here (its side streams joined st): the caller may reduce them now
                if (done != nullptr) done(user, c.index);
            }
            cur = nxt;
            which ^= 1;
        } else if (ly.kind == CNF_LAYER_FACTOR) {
            const Boundary& b = p.boundaries[bi--];
            float* prev = buf[which];
            launch_map_scatter(cur, prev, nullptr, T + b.dev_keep_src, b.n_next, b.n_next, b.n_cur, B, st);
            launch_map_scatter(dzy, prev, T + b.dev_fac_orig, T + b.dev_fac_src, b.n_fac, nuv, b.n_cur, B, st);
            cur = prev;
            which ^= 1;
        }
    }
    // the last split layers (the older first)
    const int last = lds_k & 1;
    flush(last);
    flush(last ^ 1);
    hchk(hipGetLastError(), "training kernel launch");
}

void coupling_layer_backward(Plan& p, int ci, const float* params, const float* u, const float* dv, float* du,
                             float g_ld, void* workspace, int B, float* dparams, hipStream_t st) {
    TExec E{p, params, dparams, (char*)workspace, p.layout(B), p.train_layout(B), B, st};
    E.inv_batch_ = -g_ld;
    p.tev_next = 0;
    if (p.n_bw > 0) launch_pack(params, p.dev_bw_map, E.at<float>(E.T.bw), (long long)p.n_bw, st);
    hchk(hipMemsetAsync(dparams, 0, (size_t)p.n_params * 4, st), "hipMemsetAsync");
    hchk(hipMemsetAsync(E.at<float>(E.T.zeros), 0, 64 * 4, st), "hipMemsetAsync");
    coupling_backward(E, p.couplings[ci], u, dv, du);
    hchk(hipGetLastError(), "training kernel launch");
}

}  // namespace cnf
