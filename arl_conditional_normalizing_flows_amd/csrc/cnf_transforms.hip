// cnf_transforms.hip — the input transforms that feed the flow (conv_cINN_base_functions.py):
// logit preprocessing / de_logitify, super-resolution down / up / residual assembly, and
// instance / renewed Gaussian noise. All elementwise or 2x2-block HBM-bound kernels, one thread
// per output element (float4-free: every output is computed from a handful of inputs).
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <string>

#include "../../include/cnf.h"
#include "cnf_device.h"

namespace cnf {

int set_error(int code, const char* msg);   // cnf_runtime.cpp (cnf_last_error)

// LogitK (cnf_kernels.h) of the fudge factor a
LogitK logit_consts(float a) {
    const double ad = a;
    const double b = (1.0 - 2.0 * ad) / (1.0 - ad);
    LogitK k;
    k.a = a;
    k.c1 = (float)((1.0 - ad) * b);
    k.lo = logf((float)(ad / (1.0 - ad)));
    const float hi = logf((float)((1.0 - ad) / ad));
    k.span = hi - k.lo;
    k.inv_bc = (float)(1.0 / (b * (1.0 - ad)));
    return k;
}

namespace {

// preprocess_dataset_class._preprocess_for_logit / _logit / _scale_logit (:198-212)
__global__ __launch_bounds__(256) void k_logit(const float* __restrict__ x, float* __restrict__ out, long long n,
                                               LogitK k, int inverse) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
        const float v = x[i];
        float r;
        if (!inverse) {
            r = logit_value(v, k);
        } else {   // de_logitify (:306-318): (logistic(v span + lo) - a) / (b (1 - a))
            const float z = v * k.span + k.lo;
            r = (1.f / (1.f + expf(-z)) - k.a) * k.inv_bc;
        }
        out[i] = r;
    }
}

// mean of the 2^L x 2^L block of `in` ([H][W][C] image) whose top-left corner is (r0, c0), as
// nested 2x2 means (down applied L times, :111-116: reduce_mean over each 2x2 block)
__device__ float nested_mean(const float* __restrict__ in, int W, int C, int r0, int c0, int c, int L) {
    if (L == 0) return in[((size_t)r0 * W + c0) * C + c];
    const int h = 1 << (L - 1);
    const float m00 = nested_mean(in, W, C, r0, c0, c, L - 1);
    const float m01 = nested_mean(in, W, C, r0, c0 + h, c, L - 1);
    const float m10 = nested_mean(in, W, C, r0 + h, c0, c, L - 1);
    const float m11 = nested_mean(in, W, C, r0 + h, c0 + h, c, L - 1);
    return ((m00 + m01) + (m10 + m11)) * 0.25f;
}

// preprocess_dataset_SR._preprocess_* (:252-273): one thread per (pixel, channel) of x
__global__ __launch_bounds__(256) void k_sr(const float* __restrict__ hi, float* __restrict__ xy, int B, int H, int W,
                                            int C, int xd, int yl, int residual) {
    const int Ho = H >> xd, Wo = W >> xd;
    const long long n = (long long)B * Ho * Wo * C;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
        const int c = (int)(e % C);
        const long long p = e / C;
        const int j = (int)(p % Wo);
        const long long q = p / Wo;
        const int i = (int)(q % Ho);
        const int b = (int)(q / Ho);
        const float* img = hi + (size_t)b * H * W * C;
        const int s = 1 << xd;
        const float x0 = nested_mean(img, W, C, i * s, j * s, c, xd);
        const int m = 1 << yl;
        const int bi = (i / m) * m, bj = (j / m) * m;   // y block of x0 containing (i, j)
        const float y = nested_mean(img, W, C, bi * s, bj * s, c, xd + yl);
        float* o = xy + (size_t)p * 2 * C;
        o[c] = residual ? x0 - y : x0;
        o[C + c] = y;
    }
}

__global__ __launch_bounds__(256) void k_down(const float* __restrict__ in, float* __restrict__ out, int B, int H,
                                              int W, int C) {
    const int Ho = H / 2, Wo = W / 2;
    const long long n = (long long)B * Ho * Wo * C;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
        const int c = (int)(e % C);
        const long long p = e / C;
        const int j = (int)(p % Wo);
        const long long q = p / Wo;
        const int i = (int)(q % Ho);
        const int b = (int)(q / Ho);
        out[e] = nested_mean(in + (size_t)b * H * W * C, W, C, 2 * i, 2 * j, c, 1);
    }
}

__global__ __launch_bounds__(256) void k_up(const float* __restrict__ in, float* __restrict__ out, int B, int H, int W,
                                            int C) {
    const int Ho = 2 * H, Wo = 2 * W;
    const long long n = (long long)B * Ho * Wo * C;
    for (long long e = (long long)blockIdx.x * 256 + threadIdx.x; e < n; e += (long long)gridDim.x * 256) {
        const int c = (int)(e % C);
        const long long p = e / C;
        const int j = (int)(p % Wo);
        const long long q = p / Wo;
        const int i = (int)(q % Ho);
        const int b = (int)(q / Ho);
        out[e] = in[(((size_t)b * H + i / 2) * W + j / 2) * C + c];
    }
}

// instance_noise (:635-654) / renew_noise (:660-676): element i of the stream offset + i
// (instance_noise_value, cnf_device.h)
__global__ __launch_bounds__(256) void k_noise(const float* __restrict__ x, float* __restrict__ out, long long n,
                                               float alpha, uint64_t seed, uint64_t offset) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        out[i] = instance_noise_value(x != nullptr ? x[i] : 0.f, x != nullptr, alpha, seed, offset + (uint64_t)i);
}

// cnf_flow_forward_noise's input preparation as a pass of its own (the first coupling layer is
// streamed): out[i] = input_prep_value of element i
__global__ __launch_bounds__(256) void k_prep(float* __restrict__ out, long long n, InputPrepArgs q) {
    for (long long i = (long long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long long)gridDim.x * 256)
        out[i] = input_prep_value(q.src[i], (int)(i % q.D), q, q.off + (uint64_t)i);
}

int grid_for(long long n) {
    long long g = (n + 255) / 256;
    return (int)(g < 1 ? 1 : (g > 65536 ? 65536 : g));
}

int finish(const char* what) {
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return set_error(CNF_E_HIP, (std::string(what) + ": " + hipGetErrorString(e)).c_str());
    return CNF_OK;
}

}  // namespace

void launch_input_prep(float* out, long long n, const InputPrepArgs& q, hipStream_t st) {
    if (n <= 0) return;
    hipLaunchKernelGGL(k_prep, dim3(grid_for(n)), dim3(256), 0, st, out, n, q);
}

}  // namespace cnf

extern "C" {

int cnf_logit(const float* x, float* out, int64_t n, float a, int inverse, void* stream) {
    if (!x || !out || n < 0 || !(a > 0.f && a < 0.5f))
        return cnf::set_error(CNF_E_INVALID, "cnf_logit: null pointer, n < 0 or a outside (0, 0.5)");
    if (n == 0) return CNF_OK;
    hipLaunchKernelGGL(cnf::k_logit, dim3(cnf::grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, out, (long long)n,
                       cnf::logit_consts(a), inverse);
    return cnf::finish("k_logit");
}

int cnf_sr_preprocess(const float* hires, float* xy, int B, int H, int W, int C, int x_down, int y_levels,
                      int residual, void* stream) {
    if (!hires || !xy || B <= 0 || H <= 0 || W <= 0 || C <= 0 || x_down < 0 || y_levels < 0 || x_down + y_levels > 8)
        return cnf::set_error(CNF_E_INVALID, "cnf_sr_preprocess: bad shape or levels");
    const int m = 1 << (x_down + y_levels);
    if (H % m || W % m) return cnf::set_error(CNF_E_INVALID, "cnf_sr_preprocess: H and W must be divisible by 2^(x_down + y_levels)");
    const long long n = (long long)B * (H >> x_down) * (W >> x_down) * C;
    hipLaunchKernelGGL(cnf::k_sr, dim3(cnf::grid_for(n)), dim3(256), 0, (hipStream_t)stream, hires, xy, B, H, W, C,
                       x_down, y_levels, residual);
    return cnf::finish("k_sr");
}

int cnf_down(const float* in, float* out, int B, int H, int W, int C, void* stream) {
    if (!in || !out || B <= 0 || H < 2 || W < 2 || C <= 0) return cnf::set_error(CNF_E_INVALID, "cnf_down: bad shape");
    const long long n = (long long)B * (H / 2) * (W / 2) * C;
    hipLaunchKernelGGL(cnf::k_down, dim3(cnf::grid_for(n)), dim3(256), 0, (hipStream_t)stream, in, out, B, H, W, C);
    return cnf::finish("k_down");
}

int cnf_up(const float* in, float* out, int B, int H, int W, int C, void* stream) {
    if (!in || !out || B <= 0 || H <= 0 || W <= 0 || C <= 0) return cnf::set_error(CNF_E_INVALID, "cnf_up: bad shape");
    const long long n = (long long)B * 4 * H * W * C;
    hipLaunchKernelGGL(cnf::k_up, dim3(cnf::grid_for(n)), dim3(256), 0, (hipStream_t)stream, in, out, B, H, W, C);
    return cnf::finish("k_up");
}

int cnf_instance_noise(const float* x, float* out, int64_t n, float alpha, uint64_t seed, uint64_t offset,
                       void* stream) {
    if (!out || n < 0) return cnf::set_error(CNF_E_INVALID, "cnf_instance_noise: null output or n < 0");
    if (n == 0) return CNF_OK;
    hipLaunchKernelGGL(cnf::k_noise, dim3(cnf::grid_for(n)), dim3(256), 0, (hipStream_t)stream, x, out, (long long)n,
                       alpha, seed, offset);
    return cnf::finish("k_noise");
}

}  // extern "C"
