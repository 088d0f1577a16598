// cnf_plan.cpp — host-side restatement of cFlow.__init__ (conv_cINN_make_model.py:1431-1695) and
// of the coupling-layer geometry (:355-498, :1087-1104, conv_cINN_base_functions.py:364-413, 501-627).
#include "cnf_plan.h"

#include <cmath>
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

}  // namespace

Plan* build_plan(const cnf_flow_desc* d) {
    require(d != nullptr, "null descriptor");
    auto P = new Plan();
    Plan& p = *P;
    try {
        p.desc = *d;
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
            }
        }

        // aux image: dense [9*cin][cout] weights + [cout] bias per grouped branch
        for (auto& c : p.couplings) {
            for (int net = 0; net < 2; net++) {
                for (auto& rb : c.net[net].rb) {
                    for (size_t bi = 0; bi < c.br.size(); bi++) {
                        const Branch& b = c.br[bi];
                        const int K = ks * ks * b.cin;
                        int64_t wo = p.n_aux;
                        p.aux_map.resize(p.aux_map.size() + (size_t)K * b.cout, -1);
                        for (size_t j = 0; j < b.in_offsets.size(); j++) {
                            const int64_t gk = rb.gk[bi][j];
                            const int in_rel = b.in_offsets[j] - b.cin_off;  // 0 in reference mode
                            for (int tap = 0; tap < ks * ks; tap++)
                                for (int ci2 = 0; ci2 < b.width; ci2++)
                                    for (int o = 0; o < b.width; o++) {
                                        int64_t dst = wo + (int64_t)(tap * b.cin + in_rel + ci2) * b.cout +
                                                      (int64_t)j * b.width + o;
                                        p.aux_map[dst] = gk + ((int64_t)tap * b.width + ci2) * b.width + o;
                                    }
                        }
                        p.n_aux += (int64_t)K * b.cout;
                        rb.aux_w.push_back(wo);
                        int64_t bo = p.n_aux;
                        for (size_t j = 0; j < b.in_offsets.size(); j++)
                            for (int o = 0; o < b.width; o++) p.aux_map.push_back(rb.gb[bi][j] + o);
                        p.n_aux += b.cout;
                        rb.aux_b.push_back(bo);
                    }
                }
            }
        }

        // k_net_lds offset tables
        require(p.n_params < (1ll << 31) && p.n_aux < (1ll << 31), "parameter image exceeds 2^31 floats");
        for (auto& c : p.couplings) {
            for (int net = 0; net < 2; net++) {
                const NetParams& np = c.net[net];
                std::vector<int> o = {(int)np.conv_in_k, (int)np.conv_in_b};
                for (const auto& rb : np.rb) {
                    for (int64_t v : {rb.ln1g, rb.ln1b, rb.conv_a_k, rb.conv_a_b, rb.ln2g, rb.ln2b, rb.ln3g, rb.ln3b,
                                      rb.conv_b_k, rb.conv_b_b})
                        o.push_back((int)std::max<int64_t>(v, 0));
                    for (size_t bi = 0; bi < c.br.size(); bi++) {
                        o.push_back((int)rb.aux_w[bi]);
                        o.push_back((int)rb.aux_b[bi]);
                    }
                }
                for (int64_t v : {np.ln_out_g, np.ln_out_b, np.conv_out_k, np.conv_out_b})
                    o.push_back((int)std::max<int64_t>(v, 0));
                c.lds_offs_per_net = (int)o.size();
                c.lds_offs.insert(c.lds_offs.end(), o.begin(), o.end());
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
