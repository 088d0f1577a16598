// cnf_toy.hip — the reference's TOYcINN dense conditional flow (BASELINE configs[0], the CPU
// plumbing configuration; TOYcINN_make_model.py:29-506) on the GPU.
//
// One thread carries one sample through all coupling layers in registers; the two dense nets of
// the current coupling layer (b: Dense(H)+LReLU, L x [Dense(H)+LReLU], Dense(u2); A: the same then
// tanh) are staged into LDS once per workgroup and read as broadcasts. fp32 throughout, exact
// LeakyReLU / tanh / exp as in the reference graph. The workload is tiny (3-dimensional points), so
// the kernel favours a simple, exact formulation over throughput.
#include <hip/hip_runtime.h>

#include <cstdint>

#include "cnf_kernels.h"

namespace cnf {

namespace {

__device__ __forceinline__ float lrelu_t(float x) { return x >= 0.f ? x : LRELU_ALPHA * x; }

// y[o] = sum_k x[k] W[k][o] + b[o] over LDS weights W [nin][nout] (row-major), b [nout];
// compile-time bounds keep x / y in registers
template <int NIN, int NOUT>
__device__ __forceinline__ void dense(const float* x, int nin, const float* W, const float* b, int nout, float* y) {
#pragma unroll
    for (int o = 0; o < NOUT; o++) y[o] = o < nout ? b[o] : 0.f;
#pragma unroll
    for (int k = 0; k < NIN; k++) {
        if (k < nin) {
            const float xk = x[k];
            const float* w = W + k * nout;
#pragma unroll
            for (int o = 0; o < NOUT; o++)
                if (o < nout) y[o] = fmaf(xk, w[o], y[o]);
        }
    }
}

// b or A net of one coupling layer on u1 (n1 inputs) -> out (n2 outputs); params at p (LDS);
// hidden width Hr <= H (H = register-array bound)
template <int H>
__device__ __forceinline__ const float* toy_net(const float* p, const float* u1, int n1, int Hr, int L, int n2,
                                                float* out) {
    float h[H], t[H];
    dense<2, H>(u1, n1, p, p + n1 * Hr, Hr, h);
    p += n1 * Hr + Hr;
#pragma unroll
    for (int o = 0; o < H; o++) h[o] = lrelu_t(h[o]);
    for (int l = 0; l < L; l++) {
        dense<H, H>(h, Hr, p, p + Hr * Hr, Hr, t);
        p += Hr * Hr + Hr;
#pragma unroll
        for (int o = 0; o < H; o++) h[o] = lrelu_t(t[o]);
    }
    float y[2];
    dense<H, 2>(h, Hr, p, p + Hr * n2, n2, y);
    out[0] = y[0];
    out[1] = y[1];
    return p + Hr * n2 + n2;
}

}  // namespace

template <int H>
__global__ __launch_bounds__(256) void k_toy(ToyArgs a) {
    extern __shared__ __attribute__((aligned(16))) float lw[];
    const int s = blockIdx.x * 256 + threadIdx.x;
    const bool valid = s < a.B;
    float u[3] = {0.f, 0.f, 0.f};
    if (valid)
        for (int c = 0; c < 3; c++) u[c] = a.u[(size_t)s * 3 + c];
    float ld = 0.f;
    for (int step = 0; step < a.nl; step++) {
        const int i = a.dir < 0 ? a.nl - 1 - step : step;   // direction -1: reverse index order (:300)
        const int j = a.order[i];
        const int t = j % 6;
        // u1 / u2 index sets of mask type t (:149-163)
        int i1[2], i2[2], n1, n2;
        if (t < 3) {
            n1 = 1;
            n2 = 2;
            i1[0] = t;
            i1[1] = 0;
            i2[0] = t == 0 ? 1 : 0;
            i2[1] = t == 2 ? 1 : 2;
        } else {
            n1 = 2;
            n2 = 1;
            i1[0] = t == 5 ? 1 : 0;
            i1[1] = t == 3 ? 1 : 2;
            i2[0] = 5 - t;   // t=3 -> 2, t=4 -> 1, t=5 -> 0
            i2[1] = 0;
        }
        // stage both nets of coupling network j
        const int n = a.net_off[j + 1] - a.net_off[j];
        __syncthreads();
        for (int e = threadIdx.x; e < n; e += 256) lw[e] = a.params[a.net_off[j] + e];
        __syncthreads();
        float u1[2] = {u[i1[0]], n1 > 1 ? u[i1[1]] : 0.f};
        float bv[2], av[2];
        const float* p = toy_net<H>(lw, u1, n1, a.H, a.L, n2, bv);
        toy_net<H>(p, u1, n1, a.H, a.L, n2, av);
        for (int k = 0; k < n2; k++) {
            const float A = tanhf(av[k]);
            const float u2 = u[i2[k]];
            if (a.dir < 0) {
                u[i2[k]] = expf(A) * u2 + bv[k];   // :380
                ld += A;                            // log det diag(exp A) (:386-387)
            } else {
                u[i2[k]] = (u2 - bv[k]) / expf(A);  // :370-375
            }
        }
    }
    if (!valid) return;
    for (int c = 0; c < 3; c++) a.v[(size_t)s * 3 + c] = u[c];
    if (a.dir < 0 && a.log_detJ) a.log_detJ[s] = ld;
    if (a.dir < 0 && a.per_sample) {
        // log_loss terms (:419-451): log N(z; 0, I_xd), -lambda_y |y - y'|_1, log_detJ
        float llz = -0.5f * (float)a.x_d * (float)LOG_2PI_D, lly = 0.f;
        for (int c = 0; c < 3; c++) {
            if (c < a.x_d)
                llz -= 0.5f * u[c] * u[c];
            else
                lly -= a.lambda_y * fabsf(u[c] - a.u[(size_t)s * 3 + c]);
        }
        a.per_sample[(size_t)s * 3 + 0] = llz;
        a.per_sample[(size_t)s * 3 + 1] = lly;
        a.per_sample[(size_t)s * 3 + 2] = ld;
    }
}

void launch_toy(const ToyArgs& a, int lds_floats, hipStream_t st) {
    const dim3 g((a.B + 255) / 256), b(256);
    const size_t lds = (size_t)lds_floats * sizeof(float);
    // the hidden width is a compile-time register-array bound (the reference uses 32)
    if (a.H == 32)
        hipLaunchKernelGGL(k_toy<32>, g, b, lds, st, a);
    else if (a.H <= 16)
        hipLaunchKernelGGL(k_toy<16>, g, b, lds, st, a);
    else if (a.H <= 32)
        hipLaunchKernelGGL(k_toy<32>, g, b, lds, st, a);
    else
        hipLaunchKernelGGL(k_toy<64>, g, b, lds, st, a);
}

}  // namespace cnf
