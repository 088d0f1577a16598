// cnf_plan.cpp — host-side restatement of cFlow.__init__ (conv_cINN_make_model.py:1431-1695) and
// of the coupling-layer geometry (:355-498, :1087-1104, conv_cINN_base_functions.py:364-413, 501-627).
#include <cstring>
#include "cnf_plan.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <functional>
#include <stdexcept>

namespace cnf {

namespace {

void require(bool ok, const std::string& msg) {
    if (!ok) throw std::invalid_argument(msg);
}

// conv_cINN_make_model.py:1553-1610 (dilation schedule; float arithmetic preserved)
void dilations_for_block(int h, int w, int ksize, std::vector<int>& cw, std::vector<int>& cb) {
    const double min_cw = std::min(h, w);
    const double min_cb = min_cw / 2.0;
    double d = 1.0, dk = ksize;
    if (dk > (min_cw + 1) / 2) {
        cw.push_back(1);
        cb.push_back(1);
        return;
    }
    int sanity = 0;
    while (dk < (min_cw + 1) / 2) {
        require(sanity < 10, "The dilation while loop ran unexpectedly many iterations.");
        cw.push_back((int)d);
        if (d < (min_cb + 1) / 2) cb.push_back((int)d);
        dk = (ksize - 1) * (dk - 1) + 1;
        d = ((dk - ksize) / (ksize - 1)) + 1;
        sanity++;
    }
}

// TF space_to_depth(2) on a per-image index image of shape (h,w,c):
// out[i, j, (di*2+dj)*c + ch] = in[2i+di, 2j+dj, ch]   (squeeze_layer :179)
std::vector<int> s2d(const std::vector<int>& in, int h, int w, int c) {
    std::vector<int> out((size_t)h * w * c);
    const int h2 = h / 2, w2 = w / 2, c4 = 4 * c;
    for (int i = 0; i < h2; i++)
        for (int j = 0; j < w2; j++)
            for (int di = 0; di < 2; di++)
                for (int dj = 0; dj < 2; dj++)
                    for (int ch = 0; ch < c; ch++)
                        out[((size_t)i * w2 + j) * c4 + (di * 2 + dj) * c + ch] =
                            in[((size_t)(2 * i + di) * w + (2 * j + dj)) * c + ch];
    return out;
}


// floats of a packed conv image and its K extent (see PackedConv); must match the pack lambda
void packed_dims(int fmt, int ks, int cin, int cout, int64_t& size, int& kpad) {
    if (fmt == PK_Q4) {
        const int G = (9 * (cin / 4) + 3) / 4;   // groups of 4 channel quads
        kpad = G * 16;
        size = (int64_t)G * 16 * 16 * ((cout + 15) / 16);
    } else if (fmt == PK_KN) {
        int ns = 16 * ((cout + 15) / 16);
        if (ns % 32 == 0) ns += 16;
        kpad = (ks * ks * cin + 3) / 4 * 4;
        size = (int64_t)kpad * ns;
    } else {
        const int ncol = (fmt == PK_TAP) ? 9 * cout : cout;
        kpad = (cin + 15) / 16 * 16;
        size = (int64_t)kpad * 16 * ((ncol + 15) / 16);
    }
}

int align16(int64_t v) { return (int)((v + 15) / 16 * 16); }
int stride8(int ch) {   // == 8 (mod 16) floats: conflict-free ds_read_b128 of channel quads
    int v = std::max(ch, 8);
    while (v % 16 != 8) v++;
    return v;
}
int stride2(int ch) {   // == 2 (mod 4) floats: conflict-free b32 reads of the tap-table path
    int v = std::max(ch, 2);
    while (v % 4 != 2) v++;
    return v;
}

// LDS image of k_net_lds for coupling c under the given conv formats; false if over 160 KiB.
bool netlds_geometry(const Coupling& c, int ci_fmt, int co_fmt, const std::vector<int>& gc_fmt, NetLdsGeom& g) {
    if (c.nk > 64 || c.dc2 > 64 || c.br.size() > 8) return false;
    for (const Branch& b : c.br)
        if (b.dil > 16) return false;
    const int64_t HW = (int64_t)c.hc * c.wc;
    g.sy = stride8(c.nk);
    g.s1 = stride8(c.nk);
    g.s2 = stride8(std::max(std::max(c.gc, c.nk), c.dc2));
    g.su = ci_fmt == PK_Q4 ? stride8(c.dc1) : stride2(c.dc1);
    g.s2r = std::max(g.s2, g.su);
    if (co_fmt == PK_TAP)   // tap-decomposed conv_out scratch (stride 16*nr+1) spans T1..T2
        g.s2r = std::max(g.s2r, 16 * ((9 * c.dc2 + 15) / 16) + (c.dc2 % 4 == 0 ? 4 : 1) - g.s1);
    int64_t wmax = 0, sz;
    int kmax = 4, kp;
    auto acc = [&](int fmt, int ks, int cin, int cout) {
        packed_dims(fmt, ks, cin, cout, sz, kp);
        wmax = std::max(wmax, sz + (cout + 3) / 4 * 4);   // the bias follows the weights in LDS
        if (fmt == PK_KN || fmt == PK_Q4) kmax = std::max(kmax, fmt == PK_Q4 ? kp / 4 : kp);   // tap / quad table
    };
    acc(ci_fmt, 3, c.dc1, c.nk);
    acc(co_fmt, 3, c.nk, c.dc2);
    if (c.R > 0) {
        acc(PK_1X1, 1, c.nk, c.nk);
        acc(PK_1X1, 1, c.gc, c.nk);
        // the grouped branches are staged together: images back to back, tables back to back
        int64_t wsum = 0;
        int ksum = 0;
        for (size_t bi = 0; bi < c.br.size(); bi++) {
            const int cin_pk = gc_fmt[bi] == PK_Q4 ? (c.br[bi].cin + 3) / 4 * 4 : c.br[bi].cin;
            packed_dims(gc_fmt[bi], 3, cin_pk, c.br[bi].cout, sz, kp);
            wsum += sz + (c.br[bi].cout + 3) / 4 * 4;
            ksum += gc_fmt[bi] == PK_Q4 ? kp / 4 : kp;
        }
        wmax = std::max(wmax, wsum);
        kmax = std::max(kmax, ksum);
    }
    // [0, 192): LN-statistics slots (8 waves x 3 doubles); [192, ...): this net's parameter-offset
    // table (2 + R*(10 + 2*nbr) + 4 ints), read from LDS so no phase waits on a global load of it
    const int64_t opn = 2 + (int64_t)c.R * (10 + 2 * (int64_t)c.br.size()) + 4;
    // ... then 16 zero bytes right below Y (k_net_lds: the 3x3 taps outside the image read them)
    int64_t off = std::max<int64_t>(512, align16(NETLDS_OTAB + 4 * opn) + 16);
    g.off_y = (int)off;
    off = align16(off + HW * g.sy * 4);
    g.off_t1 = (int)off;
    off = align16(off + HW * g.s1 * 4);   // T1 and T2 contiguous (tap scratch)
    g.off_t2 = (int)off;
    off = align16(off + HW * g.s2r * 4);
    g.off_w = (int)off;
    off = align16(off + wmax * 4);
    g.off_k = (int)off;
    off = align16(off + (int64_t)kmax * 4);
    // images of at most 4 16-pixel subtiles leave k_net_lds waves idle: their convs split K over the
    // waves and sum the slices through two alternating LDS buffers of (waves - 1) x 5 blocks x 1 KiB
    g.off_ks = 0;
    if ((HW + 15) / 16 <= 4) {
        g.off_ks = (int)off;
        off = align16(off + 2LL * 7 * 5 * 1024);
    }
    g.bytes = (int)std::min<int64_t>(off, 1 << 30);
    return off <= 160 * 1024;
}
}  // namespace

#ifndef CNF_AUTO_GENERIC
#define CNF_AUTO_GENERIC 6   // (diagnostic builds: 2 / 4 to A/B the two kernels)
#endif
Plan* build_plan(const cnf_flow_desc* d) {
    require(d != nullptr, "null descriptor");
    auto P = new Plan();
    Plan& p = *P;
    try {
        p.desc = *d;
        p.opts = parse_options(d->debug_options);
        // Images of 64 x 64 and above (cfg4, cfg5): generic k_pw / k_gc instantiations unless GENERIC is
        // given. Their shape-specialised bf16x6 instantiations gave intermittent differences on the
        // ragged-batch tests (cfg5 B = 64: 3 of 6 runs, 1e-2 in zy; cfg4 B = 32 once, 3e-4), the generic
        // ones none in 8 (profiles/sessions/r6_cfg5b.sh). The cause is open;
        // the 32 x 32 and smaller images' instantiations (cfg2, cfg3, ref_default) passed every run.
        if ((int64_t)d->io_h * d->io_w >= 64 * 64 &&
            !(d->debug_options != nullptr && std::strstr(d->debug_options, "GENERIC=") != nullptr))
            p.opts.generic |= CNF_AUTO_GENERIC;
        p.desc.debug_options = nullptr;   // (the caller's string: not kept)
        const int nb = d->num_blocks;
        require(nb > 0 && d->squeeze_factor_block_list && d->resnext_block_list && d->num_kernels_list &&
                    d->cardinality_list,
                "squeeze_factor_block_list, ResNeXt_block_list, num_kernels_list, and cardinality_list must all have the same length.");
        p.sfbl.assign(d->squeeze_factor_block_list, d->squeeze_factor_block_list + nb);
        p.rbl.assign(d->resnext_block_list, d->resnext_block_list + nb);
        p.nkl.assign(d->num_kernels_list, d->num_kernels_list + nb);
        p.cl.assign(d->cardinality_list, d->cardinality_list + nb);
        const int H = d->io_h, W = d->io_w, D = d->io_d, ks = d->ksize;
        require(H > 0 && W > 0 && D > 0 && d->x_d > 0 && d->x_d < D, "invalid io_shape / x_d");
        require(!(H % 2) && !(W % 2), "The model input and output must have spatial dimensions divisible by 2.");
        for (int nk : p.nkl) require(!(nk % 2), "The number of kernels in each layer must be divisible by 2.");
        for (int c : p.cl) require(!(c % 2), "The cardinality in each layer must be divisible by 2.");
        for (int s : p.sfbl) require(s == 0 || s == 1, "The only allowed entries in squeeze_factor_block_list are 0 and 1.");
        require(ks == 3, "only ksize=3 is implemented on the GPU path");
        require(d->group_mode == CNF_GROUP_REFERENCE || d->group_mode == CNF_GROUP_INTENDED, "unknown group_mode");

        // scale schedule :1493-1518
        std::vector<int> scale, npf;
        int scale_flag = 0, nprev = 0;
        for (int i = 0; i < nb; i++) {
            int s = (i == 0) ? 0 : p.sfbl[i - 1];
            if (!scale_flag) {
                scale.push_back(1);
                scale_flag = 1;
            } else {
                scale.push_back((1 << s) * scale.back());
            }
            nprev += s;
            npf.push_back(nprev);
        }
        std::vector<int> bh(nb), bw(nb), bd(nb);
        for (int i = 0; i < nb; i++) {  // :1521-1536
            require(!(H % (scale[i] * 2)) && !(W % (scale[i] * 2)),
                    "The cumulative scale (multiplied by 2 because the checkerboard-masked u/v are halved in spatial dimensions) must divide evenly into the original i/o spatial dimensions. This failed at block " +
                        std::to_string(i));
            bh[i] = H / scale[i];
            bw[i] = W / scale[i];
            bd[i] = D * scale[i];
        }
        std::vector<std::vector<int>> dil_cw(nb), dil_cb(nb);
        for (int i = 0; i < nb; i++) {
            if (d->dilations) {
                dilations_for_block(bh[i], bw[i], ks, dil_cw[i], dil_cb[i]);
                double nkc = (double)p.nkl[i] / p.cl[i];
                for (int dd : dil_cw[i])
                    require(std::fmod(nkc, (double)dd) == 0.0,
                            "The ratio (number of kernels / cardinality) must be evenly divisible by each dilation factor used in that coupling block. This failed in coupling block " +
                                std::to_string(i) + ".");
            } else {
                dil_cw[i] = {1};
                dil_cb[i] = {1};
            }
        }

        // layer list :1636-1689
        int ci = 0;
        for (int i = 0; i < nb; i++) {
            for (int m = 0; m < 4; m++) {
                Coupling c;
                c.index = ci;
                c.block = i;
                c.H = bh[i];
                c.W = bw[i];
                c.D = bd[i];
                c.mask = m;
                c.mask_c = (m == 0) ? 1 : (m == 1) ? 0 : (m == 2) ? 3 : 2;
                require(!(c.H % 2) && !(c.W % 2), "u/v must have spatial dimensions divisible by 2.");
                c.nk = (m < 2) ? p.nkl[i] / 2 : p.nkl[i];
                c.card = p.cl[i];
                c.R = p.rbl[i];
                if (m < 2) {
                    c.hc = c.H / 2;
                    c.wc = c.W / 2;
                    c.dc1 = 2 * c.D;
                } else {
                    c.hc = c.H;
                    c.wc = c.W;
                    c.dc1 = (m == 2) ? (c.D + 1) / 2 : c.D / 2;
                }
                if (c.D % 2 && m == 2)
                    c.dc2 = c.dc1 - 1;
                else if (c.D % 2 && m == 3)
                    c.dc2 = c.dc1 + 1;
                else
                    c.dc2 = c.dc1;
                require(c.dc1 > 0 && c.dc2 > 0, "coupling layer with an empty half (io depth too small)");
                c.dils = (m < 2) ? dil_cb[i] : dil_cw[i];
                int off = 0;
                for (int dd : c.dils) {
                    Branch b;
                    b.dil = dd;
                    double nb_ch = std::floor((double)c.nk / dd);  // nk // d (float floor-div)
                    if (c.card == 1) {
                        b.width = (int)nb_ch;
                        b.in_offsets = {0};
                        b.cin_off = 0;
                        b.cin = b.width;
                        b.cout = b.width;
                    } else {
                        require(std::fmod(nb_ch, (double)c.card) == 0.0, "assert not nb_channels % cardinality");
                        b.width = (int)std::floor(nb_ch / c.card);
                        require(b.width > 0, "zero-width group (nk / dilation < cardinality): the reference would build a 0-filter Conv2D");
                        b.cout = c.card * b.width;
                        if (d->group_mode == CNF_GROUP_REFERENCE) {
                            for (int j = 0; j < c.card; j++) b.in_offsets.push_back((c.card - 1) * b.width);
                            b.cin_off = (c.card - 1) * b.width;
                            b.cin = b.width;
                        } else {
                            for (int j = 0; j < c.card; j++) b.in_offsets.push_back(j * b.width);
                            b.cin_off = 0;
                            b.cin = c.card * b.width;
                        }
                    }
                    b.out_off = off;
                    off += b.cout;
                    c.br.push_back(b);
                }
                c.gc = off;
                Layer L;
                L.kind = CNF_LAYER_COUPLING;
                L.ci = ci;
                L.h = bh[i];
                L.w = bw[i];
                L.d = bd[i];
                L.block = i;
                p.layers.push_back(L);
                p.couplings.push_back(c);
                ci++;
            }
            if (p.sfbl[i] == 1) {
                Layer s;
                s.kind = CNF_LAYER_SQUEEZE;
                s.h = bh[i];
                s.w = bw[i];
                s.d = bd[i];
                s.block = i;
                p.layers.push_back(s);
                Layer f = s;
                f.kind = CNF_LAYER_FACTOR;
                f.npf = npf[i];
                p.layers.push_back(f);
            }
        }

        // canonical parameter table (Keras order; see oracle/cflow_np.py param_specs)
        auto add = [&](const std::string& name, std::vector<int> shape) -> int64_t {
            ParamTensor t;
            t.name = name;
            t.offset = p.n_params;
            t.shape = shape;
            p.n_params += t.size();
            p.params.push_back(t);
            return t.offset;
        };
        const bool ln = d->layer_norm != 0;
        for (auto& c : p.couplings) {
            for (int net = 0; net < 2; net++) {
                NetParams& np = c.net[net];
                std::string pre = "c" + std::to_string(c.index) + (net == 0 ? ".A" : ".b");
                np.lo = p.n_params;
                np.conv_in_k = add(pre + ".conv_in.kernel", {ks, ks, c.dc1, c.nk});
                np.conv_in_b = add(pre + ".conv_in.bias", {c.nk});
                const int nhw = c.hc * c.wc;
                for (int r = 0; r < c.R; r++) {
                    RBParams rb;
                    std::string q = pre + ".rb" + std::to_string(r);
                    if (ln) {
                        rb.ln1g = add(q + ".ln1.gamma", {nhw * c.nk});
                        rb.ln1b = add(q + ".ln1.beta", {nhw * c.nk});
                    }
                    rb.conv_a_k = add(q + ".conv_a.kernel", {1, 1, c.nk, c.nk});
                    rb.conv_a_b = add(q + ".conv_a.bias", {c.nk});
                    if (ln) {
                        rb.ln2g = add(q + ".ln2.gamma", {nhw * c.nk});
                        rb.ln2b = add(q + ".ln2.beta", {nhw * c.nk});
                    }
                    rb.gk.resize(c.br.size());
                    rb.gb.resize(c.br.size());
                    for (size_t bi = 0; bi < c.br.size(); bi++) {
                        const Branch& b = c.br[bi];
                        for (size_t j = 0; j < b.in_offsets.size(); j++) {
                            std::string g = q + ".gc.d" + std::to_string(bi) + ".g" + std::to_string(j);
                            rb.gk[bi].push_back(add(g + ".kernel", {ks, ks, b.width, b.width}));
                            rb.gb[bi].push_back(add(g + ".bias", {b.width}));
                        }
                    }
                    if (ln) {
                        rb.ln3g = add(q + ".ln3.gamma", {nhw * c.gc});
                        rb.ln3b = add(q + ".ln3.beta", {nhw * c.gc});
                    }
                    rb.conv_b_k = add(q + ".conv_b.kernel", {1, 1, c.gc, c.nk});
                    rb.conv_b_b = add(q + ".conv_b.bias", {c.nk});
                    np.rb.push_back(rb);
                }
                if (ln) {
                    np.ln_out_g = add(pre + ".ln_out.gamma", {nhw * c.nk});
                    np.ln_out_b = add(pre + ".ln_out.beta", {nhw * c.nk});
                }
                np.conv_out_k = add(pre + ".conv_out.kernel", {ks, ks, c.nk, c.dc2});
                np.conv_out_b = add(pre + ".conv_out.bias", {c.dc2});
                if (net == 0) np.tanh_w = add(pre + ".tanh_scale.w", {});
                np.hi = p.n_params;
            }
        }

        // conv formats and which layers run the whole-net-in-LDS kernel (CNF_NETLDS=0 disables):
        // prefer PK_Q4 for its 3x3 convs (channel-quad ds_read_b128 A reads), fall back to PK_KN
        // when the Q4 images do not fit the 160 KiB LDS image, else stream the layer.
        {
            const bool allow = p.opts.netlds != 0, allow_gc = p.opts.gc != 0;
            for (auto& c : p.couplings) {
                const int tapco = 9 * c.dc2 <= 64 ? PK_TAP : PK_KN;
                c.ci_fmt = PK_KN;
                c.co_fmt = tapco;
                c.gc_fmt.assign(c.br.size(), PK_KN);
                c.use_lds = false;
                if (!allow) continue;
                const int ci9 = c.dc1 % 4 == 0 ? PK_Q4 : PK_KN;
                // conv_out: the tap-decomposed form (1x1 GEMM to 9*dc2 columns, computed in 32-column
                // chunks, + a 9-point shifted sum) when it needs fewer MFMAs than the quad-packed 3x3
                // (ceil(nk/16) * ceil(9 dc2/16) against ceil(9 nk/16) * ceil(dc2/16) 16x16 blocks)
                const int tap_cost = (c.nk + 15) / 16 * ((9 * c.dc2 + 15) / 16);
                const int q4_cost = (9 * c.nk + 15) / 16 * ((c.dc2 + 15) / 16);
                const bool tap = tap_cost < q4_cost;
                const int coq = c.nk % 4 == 0 ? PK_Q4 : PK_KN;
                std::vector<int> gc9;
                for (const Branch& b : c.br) gc9.push_back(b.cin % 4 == 0 && b.cin_off % 4 == 0 ? PK_Q4 : PK_KN);
                NetLdsGeom g;
                int co9 = tap ? PK_TAP : coq;
                bool fit = netlds_geometry(c, ci9, co9, gc9, g);
                if (!fit && co9 == PK_TAP) {   // the tap scratch did not fit: quad-packed conv_out
                    co9 = coq;
                    fit = netlds_geometry(c, ci9, co9, gc9, g);
                }
                if (fit) {
                    c.ci_fmt = ci9;
                    c.co_fmt = co9;
                    c.gc_fmt = gc9;
                    c.use_lds = true;
                } else if (netlds_geometry(c, PK_KN, tapco, c.gc_fmt, g)) {
                    c.use_lds = true;
                }
                if (c.use_lds) c.lds = g;
            }
            // streamed layers: the grouped stage as k_gc launches. Each group of branches gets the first
            // tile that fits the LDS and staging budgets: full-width row tiles of 256 pixels, then 2-D
            // tiles (TW = 64 .. 8 columns, W % TW == 0) of 256, 128, 64 pixels. The branches are taken
            // in order of dilation and added to the current group while it still fits, else they open
            // a new group; a branch that fits no tile on its own is left out (tap mode when its
            // dilation is >= 4 and its im2col row fits, k_conv<3> otherwise).
            for (auto& c : p.couplings) {
                c.gcg.clear();
                c.gc_fused = false;
                if (c.use_lds || c.R == 0 || c.br.empty() || c.br.size() > (size_t)GC_MAXBR || !allow_gc) continue;
                // band geometry of a group at tile TH x TW: one band per branch, nblk blocks of
                // (TH + 2 dil) x (TW + 2 dil) stacked by rows (nblk > 1 / dil_eff: polyphase tiles)
                auto fit_geo = [&](const std::vector<int>& sel, int TH, int TW, int dil_eff, int nblk,
                                   Coupling::GcGroup& out, int nw = GC_NW_SPEC) -> bool {
                    int64_t off = 512;   // [256, 384): per-image LN table
                    std::vector<GcBranch> gb;
                    for (int bi : sel) {
                        const Branch& b = c.br[bi];
                        GcBranch g{};
                        g.cin_off = b.cin_off;
                        g.cin = b.cin;
                        g.cinp = (b.cin + 3) / 4 * 4;
                        g.cout = b.cout;
                        g.out_off = b.out_off;
                        g.opcs = c.gc;
                        g.dil = dil_eff > 0 ? dil_eff : b.dil;
                        // bf16x6 contraction (cnf_stream.hip k_gc): the band holds S bf16 channels per pixel
                        // and plane (2, 4, or a multiple of 8: K = 9 S in 32-deep steps, G of them)
                        g.S = b.cin <= 2 ? 2 : b.cin <= 4 ? 4 : (b.cin + 7) / 8 * 8;
                        g.G = (9 * g.S + 31) / 32;
                        g.BW = TW + 2 * g.dil;
                        g.BH = nblk * (TH + 2 * g.dil);
                        // staged band units per pixel: channel quads up to S (S = 2: one pair); the quads
                        // past the window (to S) are staged as zeros. Exact umulhi division for x < 2^16
                        const int cpq = std::max(1, g.S / 4);
                        g.cpq_mag = cpq == 1 ? 0u : (uint32_t)((((uint64_t)1 << 32) + cpq - 1) / cpq);
                        g.bw_mag = (uint32_t)((((uint64_t)1 << 32) + g.BW - 1) / g.BW);
                        if ((int64_t)g.BH * g.BW * cpq >= (1 << 16)) return false;
                        if (b.cout > 64) return false;
                        g.w_off = (int)off;   // the weights' three bf16 planes: 1 KiB per (K step, plane, 16 outputs)
                        off = align16(off + (int64_t)g.G * 3 * ((b.cout + 15) / 16) * 1024);
                        g.q_off = (int)off;   // per K octet: up to 4 band offsets (int4)
                        off = align16(off + 64LL * g.G);
                        g.b_off = (int)off;   // biases (read from LDS in the epilogue: no global load there)
                        off = align16(off + 4LL * g.cout);
                        gb.push_back(g);
                    }
                    // the bands (three planes of BH x BW x S bf16 per branch), twice: the next image is
                    // staged while the current one is computed
                    const int64_t band0 = off;
                    int64_t quads = 0;   // staged band units: at most 128 per wave (2 per thread)
                    for (GcBranch& g : gb) {
                        g.band_off = (int)off;
                        off = align16(off + 3 * align16((int64_t)g.BH * g.BW * g.S * 2));
                        quads += (int64_t)g.BH * g.BW * std::max(1, g.S / 4);
                    }
                    const int64_t band_bytes = off - band0;
                    off += band_bytes;
                    // nw < 16: 16 / nw workgroups share a CU, so its LDS
                    if (off > gc_lds_budget(nw) || quads > gc_stage_units(nw)) return false;
                    out.nw = nw;
                    out.br = sel;
                    out.gcb = gb;
                    out.TH = TH;
                    out.TW = TW;
                    out.tiles_x = c.wc / TW;
                    out.tiles_y = (c.hc + TH - 1) / TH;
                    out.lds = (int)off;
                    out.band_bytes = (int)band_bytes;
                    out.TP = TH * TW;
                    return true;
                };
                auto fit = [&](const std::vector<int>& sel, int TW, int TP, Coupling::GcGroup& out) -> bool {
                    const int TH = std::max(1, std::min(c.hc, TP / TW));   // TP-pixel tiles
                    if (!fit_geo(sel, TH, TW, 0, 1, out)) return false;
                    out.TP = TP;
                    return true;
                };
                auto fit_any = [&](const std::vector<int>& sel, Coupling::GcGroup& out) -> bool {
                    if (c.wc <= 128 && fit(sel, c.wc, 256, out)) return true;
                    for (int TP : {256, 128, 64})
                        for (int TW : {64, 32, 16, 8})
                            if (TW < c.wc && c.wc % TW == 0 && TW <= TP && fit(sel, TW, TP, out)) return true;
                    return false;
                };
                // a large dilation that does not fit the current group opens a group of its own
                // (cfg5: 485 -> 437 ms/step against tap mode)
                std::vector<int> order;
                for (size_t bi = 0; bi < c.br.size(); bi++) order.push_back((int)bi);
                std::stable_sort(order.begin(), order.end(), [&](int x, int y) { return c.br[x].dil < c.br[y].dil; });
                Coupling::GcGroup cur;
                bool have = false;
                for (int bi : order) {
                    Coupling::GcGroup g;
                    // a large dilation joins the current group only at the group's own tile (shrinking
                    // the tile for its halo costs more than a launch of its own)
                    const bool tap_able = c.br[bi].dil >= 4 && ks == 3 && 9 * c.br[bi].cin <= 128 && c.br[bi].cout <= 64;
                    if (have) {
                        std::vector<int> sel = cur.br;
                        sel.push_back(bi);
                        if (tap_able ? fit(sel, cur.TW, cur.TP, g) : fit_any(sel, g)) {
                            cur = g;
                            continue;
                        }
                    }
                    if (fit_any({bi}, g)) {
                        if (have) c.gcg.push_back(cur);
                        cur = g;
                        have = true;
                    }
                }
                if (have) c.gcg.push_back(cur);
                // a group of one large-dilation branch on polyphase tiles when its phase grids are whole
                // (H, W divisible by the dilation): bands of (TH+2) x (TW+2) per grid instead of
                // (TH + 2d) x (TW + 2d) (cfg5's dilation-16 branch: 400 staged pixels per 256 outputs
                // instead of 1920 per 128); debug option LAYOUT without bit 4: none
                const bool poly = (p.opts.layout & 4) != 0;
                for (auto& gg : c.gcg) {
                    if (!poly || gg.br.size() != 1) continue;
                    const Branch& b = c.br[gg.br[0]];
                    const int d = b.dil;
                    if (d < 4 || c.hc % d || c.wc % d) continue;
                    const int hs = c.hc / d, wsb = c.wc / d;
                    if (wsb > 256 || hs * wsb < 1) continue;
                    // tiles of TP pixels: nbk whole grids, or TH-row slices of one grid
                    auto tile_for = [&](int TP, int& nbk, int& TH, int& tpp) {
                        nbk = 1;
                        TH = hs;
                        tpp = 1;
                        if (hs * wsb <= TP) {
                            while (nbk * 2 * hs * wsb <= TP && (d * d) % (nbk * 2) == 0) nbk *= 2;
                        } else {
                            TH = std::max(1, TP / wsb);
                            while (hs % TH) TH--;
                            tpp = hs / TH;
                        }
                    };
                    // four 4-wave workgroups per CU when the band is small (these branches have little
                    // MFMA work per image: their time is per-image latency, which co-resident
                    // workgroups hide; tiles down to 128 pixels for it), else one 16-wave workgroup
                    Coupling::GcGroup g;
                    int nbk = 1, TH = hs, tpp = 1;
                    bool ok = false;
                    for (int TP : {256, 128}) {
                        tile_for(TP, nbk, TH, tpp);
                        if ((ok = fit_geo(gg.br, TH, wsb, 1, nbk, g, 4))) break;
                    }
                    if (!ok) {
                        tile_for(256, nbk, TH, tpp);
                        ok = fit_geo(gg.br, TH, wsb, 1, nbk, g);
                    }
                    if (!ok) continue;
                    g.ps = d;
                    // little work per image: the next image's band load is a whole memory round trip
                    // per image unless several are in flight (4 images: 32 VGPRs at 2 quads per thread)
                    g.pd = g.nw == 4 ? 4 : 1;
                    g.nbk = nbk;
                    g.tpp = tpp;
                    g.tiles_x = 1;
                    g.tiles_y = (d * d / nbk) * tpp;
                    gg = g;
                }
                c.gc_fused = !c.gcg.empty();
                for (const auto& g : c.gcg)
                    for (int bi : g.br) c.gc_fmt[bi] = PK_Q4;
            }
            // streamed layers: t1 as one dense sub-tensor per consumer of it (Coupling::t1_map): each
            // k_gc group (and each branch launched on its own) reads only its windows, 16-byte aligned,
            // instead of a few channels out of every 256-byte pixel. conv_a runs as k_pw for it (CNF_PW=0
            // selects k_conv1, which stores the plain layout), and no branch may be left to k_conv<3>
            // (plain layout only); debug option LAYOUT without bit 1: the plain layout
            const bool allow_c = p.opts.pw != 0 && (p.opts.layout & 1) != 0;
            constexpr int tap_dmin = 4;   // as the packing below
            for (auto& c : p.couplings) {
                c.t1_cs = c.nk;
                c.t1_compact = false;
                c.t1_used = 0;
                c.t1_off.clear();
                c.t1_pcs.clear();
                c.t1_map.clear();
                for (const Branch& b : c.br) {
                    c.t1_off.push_back(b.cin_off);
                    c.t1_pcs.push_back(c.nk);
                    for (int ch = b.cin_off; ch < b.cin_off + b.cin && ch < 64; ch++) c.t1_used |= 1ull << ch;
                }
                for (auto& g : c.gcg)
                    for (size_t k = 0; k < g.br.size(); k++) {
                        g.gcb[k].cin_off = c.br[g.br[k]].cin_off;
                        g.gcb[k].pcs = c.nk;
                    }
                if (c.use_lds || c.R == 0 || c.br.empty() || c.nk > 64 || !allow_c) continue;
                // consumers: the k_gc groups, then every other branch (k_pw tap mode) on its own
                std::vector<std::vector<int>> units;
                for (const auto& g : c.gcg) units.push_back(g.br);
                bool ok = true;
                for (size_t bi = 0; bi < c.br.size(); bi++) {
                    if (c.in_gc((int)bi)) continue;
                    const Branch& b = c.br[bi];
                    ok = ok && ks == 3 && 9 * b.cin <= 128 && b.cout <= 64 && b.dil >= tap_dmin;
                    units.push_back({(int)bi});
                }
                if (!ok) continue;
                // every window of a unit at the next 16-byte boundary (in channel order), so each
                // branch's quads stay aligned; windows of one unit must not overlap (one channel, one
                // place), nor may two units share a channel
                std::vector<std::vector<std::pair<int, int>>> uw;   // per unit: (cin_off, branch) sorted
                std::vector<int> ucs;
                uint64_t seen = 0;
                int total = 0;
                for (const auto& u : units) {
                    std::vector<std::pair<int, int>> ws;
                    for (int bi : u) ws.push_back({c.br[bi].cin_off, bi});
                    std::sort(ws.begin(), ws.end());
                    uint64_t m = 0;
                    int cs = 0;
                    for (const auto& wv : ws) {
                        const Branch& b = c.br[wv.second];
                        for (int ch = b.cin_off; ch < b.cin_off + b.cin; ch++) {
                            ok = ok && ((m | seen) >> ch & 1ull) == 0;
                            m |= 1ull << ch;
                        }
                        cs += (b.cin + 3) / 4 * 4;
                    }
                    seen |= m;
                    uw.push_back(ws);
                    ucs.push_back(cs);
                    total += cs;
                }
                if (!ok || (units.size() == 1 && total >= c.nk)) continue;
                const int hw = c.hc * c.wc;
                c.t1_compact = true;
                c.t1_cs = total;
                c.t1_map.assign(128, -1);
                int base = 0;   // floats from the image start to the sub-tensor
                for (size_t u = 0; u < units.size(); u++) {
                    const int cs = ucs[u];
                    int wo = 0;
                    for (const auto& wv : uw[u]) {
                        const Branch& b = c.br[wv.second];
                        for (int ch = b.cin_off; ch < b.cin_off + b.cin; ch++) {
                            c.t1_map[2 * ch] = base + wo + (ch - b.cin_off);
                            c.t1_map[2 * ch + 1] = cs;
                        }
                        c.t1_off[wv.second] = base + wo;
                        c.t1_pcs[wv.second] = cs;
                        wo += (b.cin + 3) / 4 * 4;
                    }
                    base += hw * cs;
                }
                for (auto& g : c.gcg)
                    for (size_t k = 0; k < g.br.size(); k++) {
                        g.gcb[k].cin_off = c.t1_off[g.br[k]];
                        g.gcb[k].pcs = c.t1_pcs[g.br[k]];
                    }
            }
        }

        // t2 split into its producers' sub-tensors when there are several (cfg4 / cfg5: k_gc groups of one
        // branch each); debug option LAYOUT without bit 2: the plain layout
        {
            const bool allow_t2 = p.opts.pw != 0 && (p.opts.layout & 2) != 0;
            constexpr int tap_dmin2 = 4;
            for (auto& c : p.couplings) {
                c.t2_mapped = false;
                c.t2_cs = c.gc;
                c.t2_off.clear();
                c.t2_pcs.clear();
                c.t2_qmap.clear();
                c.t2_bmap.clear();
                for (const Branch& b : c.br) {
                    c.t2_off.push_back(b.out_off);
                    c.t2_pcs.push_back(c.gc);
                }
                if (c.use_lds || c.R == 0 || c.br.empty() || !allow_t2 || c.gc % 4 != 0 || c.gc > 128) continue;
                std::vector<std::vector<int>> units;
                for (const auto& g : c.gcg) units.push_back(g.br);
                bool ok = true;
                for (size_t bi = 0; bi < c.br.size(); bi++) {
                    const Branch& b = c.br[bi];
                    ok = ok && b.out_off % 4 == 0 && b.cout % 4 == 0;
                    if (c.in_gc((int)bi)) continue;
                    ok = ok && ks == 3 && 9 * b.cin <= 128 && b.cout <= 64 && b.dil >= tap_dmin2;
                    units.push_back({(int)bi});
                }
                if (!ok || units.size() < 2) continue;
                const int hw = c.hc * c.wc;
                std::vector<int> ust, ucs;
                int total = 0;
                for (const auto& u : units) {
                    int lo = 1 << 30, hi = 0, sum = 0;
                    for (int bi : u) {
                        lo = std::min(lo, c.br[bi].out_off);
                        hi = std::max(hi, c.br[bi].out_off + c.br[bi].cout);
                        sum += c.br[bi].cout;
                    }
                    ok = ok && sum == hi - lo;   // the unit's slices are one channel range
                    ust.push_back(lo);
                    ucs.push_back(hi - lo);
                    total += hi - lo;
                }
                if (!ok || total != c.gc) continue;
                c.t2_mapped = true;
                c.t2_cs = total;
                c.t2_qmap.assign((size_t)2 * (c.gc / 4), -1);
                c.t2_bmap.assign(c.br.size(), std::vector<int>(128, -1));
                int base = 0;
                for (size_t u = 0; u < units.size(); u++) {
                    for (int ch = ust[u]; ch < ust[u] + ucs[u]; ch += 4) {
                        c.t2_qmap[2 * (ch / 4)] = base + (ch - ust[u]);
                        c.t2_qmap[2 * (ch / 4) + 1] = ucs[u];
                    }
                    for (int bi : units[u]) {
                        const Branch& b = c.br[bi];
                        c.t2_off[bi] = base + (b.out_off - ust[u]);
                        c.t2_pcs[bi] = ucs[u];
                        for (int j = 0; j < b.cout; j++) {
                            c.t2_bmap[bi][2 * j] = c.t2_off[bi] + j;
                            c.t2_bmap[bi][2 * j + 1] = ucs[u];
                        }
                    }
                    base += hw * ucs[u];
                }
                for (auto& g : c.gcg)
                    for (size_t k = 0; k < g.br.size(); k++) {
                        g.gcb[k].out_off = c.t2_off[g.br[k]];
                        g.gcb[k].opcs = c.t2_pcs[g.br[k]];
                    }
            }
        }

        // kernel image (aux): every conv's weights + bias packed in its kernel's LDS layout
        auto pack = [&](PackedConv& pc, int fmt, int cin, int cout, const std::function<int64_t(int, int)>& src,
                        const std::function<int64_t(int)>& bsrc) {
            pc.fmt = fmt;
            pc.cin = cin;
            pc.cout = cout;
            pc.w = p.n_aux;
            if (fmt == PK_Q4) {
                // K = 9*cin as a list of channel quads qd = tap*(cin/4) + cq (k = tap*cin + 4cq + s);
                // image [g][q][j][s] with qd = 4g + q
                const int cpq = cin / 4, nq = 9 * cpq;
                pc.nr = (cout + 15) / 16;
                pc.ns = 16 * pc.nr;
                pc.G = (nq + 3) / 4;
                pc.kpad = pc.G * 16;
                pc.size = (int64_t)pc.G * 16 * pc.ns;
                for (int g = 0; g < pc.G; g++)
                    for (int q = 0; q < 4; q++)
                        for (int j = 0; j < pc.ns; j++)
                            for (int s4 = 0; s4 < 4; s4++) {
                                const int qd = 4 * g + q;
                                int64_t v = -1;
                                if (qd < nq && j < cout) {
                                    const int tap = qd / cpq, cq = qd - tap * cpq;
                                    v = src(tap * cin + 4 * cq + s4, j);
                                }
                                p.aux_map.push_back(v);
                            }
            } else if (fmt == PK_KN) {
                const int K = ks * ks * cin;
                pc.nr = (cout + 15) / 16;
                pc.ns = 16 * pc.nr;
                if (pc.ns % 32 == 0) pc.ns += 16;
                pc.kpad = (K + 3) / 4 * 4;
                pc.size = (int64_t)pc.kpad * pc.ns;
                for (int k = 0; k < pc.kpad; k++)
                    for (int n = 0; n < pc.ns; n++) p.aux_map.push_back((k < K && n < cout) ? src(k, n) : -1);
            } else {
                const int ncol = (fmt == PK_TAP) ? 9 * cout : cout;
                pc.nr = (ncol + 15) / 16;
                pc.ns = 16 * pc.nr;
                pc.G = (cin + 15) / 16;
                pc.kpad = pc.G * 16;
                pc.size = (int64_t)pc.G * 16 * pc.ns;
                for (int g = 0; g < pc.G; g++)
                    for (int q = 0; q < 4; q++)
                        for (int j = 0; j < pc.ns; j++)
                            for (int s4 = 0; s4 < 4; s4++) {
                                const int c = 16 * g + 4 * q + s4;
                                p.aux_map.push_back((c < cin && j < ncol) ? src(c, j) : -1);
                            }
            }
            p.n_aux += pc.size;
            pc.b = p.n_aux;
            const int bpad = (cout + 3) / 4 * 4;
            for (int n = 0; n < bpad; n++) p.aux_map.push_back(n < cout ? bsrc(n) : -1);
            p.n_aux += bpad;
        };
        // dense backward image: every conv as [taps][cin][cout] + [cout] bias (training kernels)
        auto dense_img = [&](PackedConv& pc, int taps, int cin, int cout, const std::function<int64_t(int, int)>& src,
                             const std::function<int64_t(int)>& bsrc) {
            pc.taps = taps;
            pc.dw = p.n_bw;
            for (int k = 0; k < taps * cin; k++)
                for (int n = 0; n < cout; n++) p.bw_map.push_back(src(k, n));
            p.n_bw += (int64_t)taps * cin * cout;
            pc.db = p.n_bw;
            for (int n = 0; n < cout; n++) p.bw_map.push_back(bsrc(n));
            p.n_bw += (cout + 3) / 4 * 4;
            for (int n = cout; n < (cout + 3) / 4 * 4; n++) p.bw_map.push_back(-1);
        };
        for (auto& c : p.couplings) {
            for (int net = 0; net < 2; net++) {
                NetParams& np = c.net[net];
                const int64_t cik = np.conv_in_k, cib = np.conv_in_b;
                const int nk = c.nk;
                pack(np.ci, c.ci_fmt, c.dc1, nk, [=](int k, int n) { return cik + (int64_t)k * nk + n; },
                     [=](int n) { return cib + n; });
                dense_img(np.ci, ks * ks, c.dc1, nk, [=](int k, int n) { return cik + (int64_t)k * nk + n; },
                          [=](int n) { return cib + n; });
                // streamed layers: conv_in for k_pw's tap mode, the HWIO kernel read as its
                // [9*dc1][nk] im2col matrix (k = tap * dc1 + c)
                // (dc1 <= 4: the im2col gathers are scalar mask-position loads, cheap only for narrow halves)
                if (!c.use_lds && ks == 3 && c.dc1 <= 4 && nk <= 64)
                    pack(np.ci_pw, PK_1X1, 9 * c.dc1, nk, [=](int k, int n) { return cik + (int64_t)k * nk + n; },
                         [=](int n) { return cib + n; });
                for (auto& rb : np.rb) {
                    const int64_t ak = rb.conv_a_k, ab = rb.conv_a_b, bk = rb.conv_b_k, bb = rb.conv_b_b;
                    pack(rb.ca, PK_1X1, nk, nk, [=](int ci2, int j) { return ak + (int64_t)ci2 * nk + j; },
                         [=](int n) { return ab + n; });
                    dense_img(rb.ca, 1, nk, nk, [=](int ci2, int j) { return ak + (int64_t)ci2 * nk + j; },
                              [=](int n) { return ab + n; });
                    for (size_t bi = 0; bi < c.br.size(); bi++) {
                        const Branch b = c.br[bi];
                        const std::vector<int64_t> gk = rb.gk[bi], gb = rb.gb[bi];
                        PackedConv pc;
                        // dense [9*cin][cout] view of the card per-group Conv2D kernels (:401-411)
                        auto dense = [=](int k, int n) -> int64_t {
                            const int tap = k / b.cin, ci2 = k - tap * b.cin;
                            const int j = n / b.width, o = n - j * b.width;
                            const int in_rel = b.in_offsets[j] - b.cin_off;
                            const int cj = ci2 - in_rel;
                            if (cj < 0 || cj >= b.width) return -1;
                            return gk[j] + ((int64_t)tap * b.width + cj) * b.width + o;
                        };
                        // PK_Q4 over cin padded to a multiple of 4 (padding channels carry zero weights)
                        const int cin_pk = c.gc_fmt[bi] == PK_Q4 ? (b.cin + 3) / 4 * 4 : b.cin;
                        pack(pc, c.gc_fmt[bi], cin_pk, b.cout,
                             [=](int k, int n) -> int64_t {
                                 const int tap = k / cin_pk, ci = k - tap * cin_pk;
                                 return ci < b.cin ? dense(tap * b.cin + ci, n) : -1;
                             },
                             [=](int n) { return gb[n / b.width] + (n % b.width); });
                        dense_img(pc, ks * ks, b.cin, b.cout, dense, [=](int n) { return gb[n / b.width] + (n % b.width); });
                        rb.gc.push_back(pc);
                        // streamed layers without k_gc: the branch as k_pw's tap mode (a 1x1 over the
                        // 9*cin im2col row, k = tap * cin + c) when the row fits (K <= 128)
                        // (dilations >= 4 only: below that the staged band's halo is cheap and k_conv<3>'s
                        // coalesced band loads beat the row's strided gathers)
                        PackedConv pw;
                        constexpr int tap_dmin = 4;
                        const bool in_gc = c.in_gc((int)bi);
                        if (!c.use_lds && !in_gc && ks == 3 && 9 * b.cin <= 128 && b.cout <= 64 && b.dil >= tap_dmin)
                            pack(pw, PK_1X1, 9 * b.cin, b.cout, dense, [=](int n) { return gb[n / b.width] + (n % b.width); });
                        rb.gpw.push_back(pw);
                    }
                    if (c.t1_compact && ln) {   // LN2 gamma/beta in t1's layout (0 on padding)
                        const int64_t hw = (int64_t)c.hc * c.wc;
                        std::vector<int64_t> at((size_t)hw * c.t1_cs, -1);   // image float -> t1 channel's param
                        for (int ch = 0; ch < 64; ch++)
                            if (c.t1_map[2 * ch] >= 0)
                                for (int64_t px = 0; px < hw; px++) at[c.t1_map[2 * ch] + px * c.t1_map[2 * ch + 1]] = px * nk + ch;
                        for (int which = 0; which < 2; which++) {
                            const int64_t src = which == 0 ? rb.ln2g : rb.ln2b;
                            (which == 0 ? rb.ln2c_g : rb.ln2c_b) = p.n_aux;
                            for (int64_t v : at) p.aux_map.push_back(v >= 0 ? src + v : -1);
                            p.n_aux += (int64_t)at.size();
                        }
                    }
                    if (c.t2_mapped && ln) {   // LN3 gamma/beta in t2's layout
                        const int64_t hw = (int64_t)c.hc * c.wc;
                        std::vector<int64_t> at((size_t)hw * c.t2_cs, -1);
                        for (int ch = 0; ch < c.gc; ch++) {
                            const int o = c.t2_qmap[2 * (ch / 4)] + ch % 4, st = c.t2_qmap[2 * (ch / 4) + 1];
                            for (int64_t px = 0; px < hw; px++) at[o + px * st] = px * c.gc + ch;
                        }
                        for (int which = 0; which < 2; which++) {
                            const int64_t src = which == 0 ? rb.ln3g : rb.ln3b;
                            (which == 0 ? rb.ln3c_g : rb.ln3c_b) = p.n_aux;
                            for (int64_t v : at) p.aux_map.push_back(v >= 0 ? src + v : -1);
                            p.n_aux += (int64_t)at.size();
                        }
                    }
                    pack(rb.cb, PK_1X1, c.gc, nk, [=](int ci2, int j) { return bk + (int64_t)ci2 * nk + j; },
                         [=](int n) { return bb + n; });
                    dense_img(rb.cb, 1, c.gc, nk, [=](int ci2, int j) { return bk + (int64_t)ci2 * nk + j; },
                              [=](int n) { return bb + n; });
                }
                const int64_t ok = np.conv_out_k, ob = np.conv_out_b;
                const int dc2 = c.dc2;
                if (c.co_fmt == PK_TAP)
                    pack(np.co, PK_TAP, nk, dc2,
                         [=](int ci2, int j) {
                             const int tap = j / dc2, o = j - tap * dc2;
                             return ok + ((int64_t)tap * nk + ci2) * dc2 + o;
                         },
                         [=](int n) { return ob + n; });
                else
                    pack(np.co, c.co_fmt, nk, dc2,
                         [=](int k, int n) { return ok + (int64_t)k * dc2 + n; },
                         [=](int n) { return ob + n; });
                dense_img(np.co, ks * ks, nk, dc2, [=](int k, int n) { return ok + (int64_t)k * dc2 + n; },
                          [=](int n) { return ob + n; });
                // the streamed kernels produce at most 64 output channels per problem
                if (!c.use_lds && c.co_fmt != PK_TAP && dc2 > 64) {
                    for (int c0 = 0; c0 < dc2; c0 += 64) {
                        const int w = std::min(64, dc2 - c0);
                        PackedConv pc;
                        pack(pc, PK_KN, nk, w, [=](int k, int n) { return ok + (int64_t)k * dc2 + c0 + n; },
                             [=](int n) { return ob + c0 + n; });
                        np.co_chunks.push_back(pc);
                    }
                }
            }
        }

        p.aux_zero = p.n_aux;   // 128 zeros (bias of the bias-free tap GEMM, up to 80 columns)
        for (int i = 0; i < 128; i++) p.aux_map.push_back(-1);
        p.n_aux += 128;

        // k_net_lds offset table (params offsets for LN gamma/beta, kernel-image offsets for convs)
        require(p.n_params < (1ll << 31) && p.n_aux < (1ll << 31), "parameter image exceeds 2^31 floats");
        for (auto& c : p.couplings) {
            for (int net = 0; net < 2; net++) {
                const NetParams& np = c.net[net];
                std::vector<int> o = {(int)np.ci.w, (int)np.ci.b};
                for (const auto& rb : np.rb) {
                    for (int64_t v : {rb.ln1g, rb.ln1b, rb.ca.w, rb.ca.b, rb.ln2g, rb.ln2b, rb.ln3g, rb.ln3b, rb.cb.w,
                                      rb.cb.b})
                        o.push_back((int)std::max<int64_t>(v, 0));
                    for (const auto& g : rb.gc) {
                        o.push_back((int)g.w);
                        o.push_back((int)g.b);
                    }
                }
                for (int64_t v : {np.ln_out_g, np.ln_out_b, np.co.w, np.co.b}) o.push_back((int)std::max<int64_t>(v, 0));
                c.lds_offs_per_net = (int)o.size();
                c.lds_offs.insert(c.lds_offs.end(), o.begin(), o.end());
            }
        }
        // fused LDS-layer backward offset table (LDSBWD_* layout: canonical LN / range offsets, dense
        // backward-image conv offsets)
        require(p.n_bw < (1ll << 31), "dense backward image exceeds 2^31 floats");
        for (auto& c : p.couplings) {
            if (!c.use_lds) continue;
            for (int net = 0; net < 2; net++) {
                const NetParams& np = c.net[net];
                std::vector<int> o = {(int)np.lo, (int)np.ci.dw, (int)np.ci.db, (int)np.ln_out_g, (int)np.ln_out_b,
                                      (int)np.co.dw, (int)np.co.db, (int)np.tanh_w, (int)np.conv_in_k, (int)np.conv_in_b,
                                      (int)np.conv_out_k, (int)np.conv_out_b};
                for (const auto& rb : np.rb) {
                    for (int64_t v : {rb.ln1g, rb.ln1b, rb.ca.dw, rb.ca.db, rb.ln2g, rb.ln2b, rb.ln3g, rb.ln3b, rb.cb.dw,
                                      rb.cb.db, rb.conv_a_k, rb.conv_a_b, rb.conv_b_k, rb.conv_b_b})
                        o.push_back((int)v);
                    for (const auto& g : rb.gc) {
                        o.push_back((int)g.dw);
                        o.push_back((int)g.db);
                    }
                }
                c.bwd_offs_per_net = (int)o.size();
                c.bwd_offs.insert(c.bwd_offs.end(), o.begin(), o.end());
            }
        }

        // squeeze/factor boundary maps. orig[i] = position in the xy layout of element i of
        // the current block layout: the forward's final restoration (:1762-1770) is the exact
        // inverse of the squeeze/factor chain, so every element returns to where it started.
        int ch = H, cw = W, cd = D;
        std::vector<int> orig((size_t)H * W * D);
        for (size_t i = 0; i < orig.size(); i++) orig[i] = (int)i;
        for (int i = 0; i < nb; i++) {
            if (p.sfbl[i] != 1) continue;
            Boundary bd;
            bd.after_block = i;
            const int n = ch * cw * cd;
            std::vector<int> ar(n);
            for (int k = 0; k < n; k++) ar[k] = k;
            std::vector<int> sq = s2d(ar, ch, cw, cd);
            const int h2 = ch / 2, w2 = cw / 2, c4 = 4 * cd, split = c4 / 2;
            std::vector<int> norig;
            for (int px = 0; px < h2 * w2; px++) {
                for (int c = 0; c < split; c++) {
                    int src = sq[(size_t)px * c4 + c];
                    bd.fac_src.push_back(src);
                    bd.fac_orig.push_back(orig[src]);
                }
                for (int c = split; c < c4; c++) {
                    int src = sq[(size_t)px * c4 + c];
                    bd.keep_src.push_back(src);
                    norig.push_back(orig[src]);
                }
            }
            bd.n_cur = n;
            bd.n_next = (int)bd.keep_src.size();
            bd.n_fac = (int)bd.fac_src.size();
            orig = norig;
            ch = h2;
            cw = w2;
            cd = split;
            p.boundaries.push_back(bd);
        }
        p.final_orig = orig;
        p.last_n = (int)orig.size();

        // device table image: [boundaries..., final_orig]
        for (auto& b : p.boundaries) {
            b.dev_keep_src = (int)p.host_table.size();
            p.host_table.insert(p.host_table.end(), b.keep_src.begin(), b.keep_src.end());
            b.dev_fac_src = (int)p.host_table.size();
            p.host_table.insert(p.host_table.end(), b.fac_src.begin(), b.fac_src.end());
            b.dev_fac_orig = (int)p.host_table.size();
            p.host_table.insert(p.host_table.end(), b.fac_orig.begin(), b.fac_orig.end());
        }
        for (auto& c : p.couplings) {
            c.dev_lds_offs = (int)p.host_table.size();
            p.host_table.insert(p.host_table.end(), c.lds_offs.begin(), c.lds_offs.end());
            if (!c.bwd_offs.empty()) {
                c.dev_bwd_offs = (int)p.host_table.size();
                p.host_table.insert(p.host_table.end(), c.bwd_offs.begin(), c.bwd_offs.end());
            }
            if (c.t1_compact) {
                c.dev_t1_map = (int)p.host_table.size();
                p.host_table.insert(p.host_table.end(), c.t1_map.begin(), c.t1_map.end());
            }
            c.dev_t2_bmap.assign(c.br.size(), -1);
            if (c.t2_mapped) {
                c.dev_t2_qmap = (int)p.host_table.size();
                p.host_table.insert(p.host_table.end(), c.t2_qmap.begin(), c.t2_qmap.end());
                for (size_t bi = 0; bi < c.br.size(); bi++) {
                    c.dev_t2_bmap[bi] = (int)p.host_table.size();
                    p.host_table.insert(p.host_table.end(), c.t2_bmap[bi].begin(), c.t2_bmap[bi].end());
                }
            }
        }
        p.dev_final_orig = (int)p.host_table.size();
        p.host_table.insert(p.host_table.end(), p.final_orig.begin(), p.final_orig.end());
    } catch (...) {
        delete P;
        throw;
    }
    return P;
}

}  // namespace cnf
