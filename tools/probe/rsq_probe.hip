// Accuracy of v_rsq_f64 alone and after one / two Newton steps, against
// 1/sqrt in long double on the host, over positive doubles spanning the
// diagonal pivots the BCR factor sees (1e-8 .. 1e12).
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <random>
#include <vector>

__global__ void rsq_kernel(const double* d, double* y0, double* y1, double* y2, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double x = d[i];
    double y = __builtin_amdgcn_rsq(x);
    y0[i] = y;
    double hy = 0.5 * x * y;
    y = fma(y, fma(-hy, y, 0.5), y);
    y1[i] = y;
    hy = 0.5 * x * y;
    y = fma(y, fma(-hy, y, 0.5), y);
    y2[i] = y;
}

int main() {
    const int n = 1 << 20;
    std::mt19937_64 rng(7);
    std::uniform_real_distribution<double> e(-8.0, 12.0), m(1.0, 10.0);
    std::vector<double> d(n), y0(n), y1(n), y2(n);
    for (auto& v : d) v = m(rng) * std::pow(10.0, e(rng));
    double *dd, *a, *b, *c;
    hipMalloc(&dd, n * 8); hipMalloc(&a, n * 8); hipMalloc(&b, n * 8); hipMalloc(&c, n * 8);
    hipMemcpy(dd, d.data(), n * 8, hipMemcpyHostToDevice);
    rsq_kernel<<<n / 256, 256>>>(dd, a, b, c, n);
    hipMemcpy(y0.data(), a, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(y1.data(), b, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(y2.data(), c, n * 8, hipMemcpyDeviceToHost);
    double e0 = 0, e1 = 0, e2 = 0;
    for (int i = 0; i < n; ++i) {
        const long double r = 1.0L / std::sqrt((long double)d[i]);
        e0 = std::fmax(e0, (double)std::fabs((y0[i] - r) / r));
        e1 = std::fmax(e1, (double)std::fabs((y1[i] - r) / r));
        e2 = std::fmax(e2, (double)std::fabs((y2[i] - r) / r));
    }
    std::printf("max rel err: rsq %.3e, +1 newton %.3e, +2 newton %.3e (ulp %.3e)\n", e0, e1, e2, 0x1p-53);
    return 0;
}
