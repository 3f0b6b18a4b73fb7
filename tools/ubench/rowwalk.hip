// Micro-benchmark: the extrema sweep's read pattern (four fp32 planes, each wave walking a strip of rows down its
// columns) with 4-byte loads (64 columns per wave) against 8- and 16-byte loads (128 / 256 columns per wave).
// Reports GB/s of plane bytes read. Build: hipcc -O3 --offload-arch=gfx950 tools/ubench/rowwalk.hip -o /tmp/rowwalk
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CHECK(x) do { hipError_t err_ = (x); if (err_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(err_), __LINE__); exit(1); } } while (0)

constexpr int kStrip = 64, kWaves = 4;

template <int V>
struct Vec;
template <> struct Vec<1> { typedef float T; };
template <> struct Vec<2> { typedef float2 T; };
template <> struct Vec<4> { typedef float4 T; };

__device__ __forceinline__ float hsum(float v) { return v; }
__device__ __forceinline__ float hsum(float2 v) { return v.x + v.y; }
__device__ __forceinline__ float hsum(float4 v) { return (v.x + v.y) + (v.z + v.w); }

// grid (W / (64 V kWaves), H / kStrip, B); each lane V consecutive columns, rows y0 .. y0 + kStrip + 1
template <int V>
__global__ __launch_bounds__(64 * kWaves) void rowwalk(const float* __restrict__ p0, const float* __restrict__ p1,
                                                       const float* __restrict__ p2, const float* __restrict__ p3,
                                                       int H, int W, float* __restrict__ out) {
    typedef typename Vec<V>::T T;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, b = blockIdx.z;
    const int c = ((blockIdx.x * kWaves + wave) * 64 + lane) * V;
    const int y0 = blockIdx.y * kStrip;
    const size_t base = (size_t)b * H * W;
    const float* g[4] = {p0 + base, p1 + base, p2 + base, p3 + base};
    float acc = 0.f;
    T r[6][4];
    auto fetch = [&](int y, T (&d)[4]) {
        const uint32_t off = (uint32_t)(min(y, H - 1) * W + c);
#pragma unroll
        for (int l = 0; l < 4; ++l) d[l] = *(const T*)(g[l] + off);
    };
#pragma unroll
    for (int k = 0; k < 6; ++k) fetch(y0 + k, r[k]);
    const int y_end = min(y0 + kStrip + 2, H);
    for (int y = y0; y < y_end; y += 6) {
#pragma unroll
        for (int k = 0; k < 6; ++k) {
#pragma unroll
            for (int l = 0; l < 4; ++l) acc += hsum(r[k][l]);
            fetch(min(y + 6 + k, y_end - 1), r[k]);
        }
    }
    out[((size_t)b * gridDim.y + blockIdx.y) * gridDim.x * 64 * kWaves + blockIdx.x * 64 * kWaves + threadIdx.x] = acc;
}

template <int V>
float run(float* const* planes, int B, int H, int W, float* out, int reps) {
    dim3 grid(W / (64 * V * kWaves), H / kStrip, B);
    hipEvent_t a, e;
    CHECK(hipEventCreate(&a));
    CHECK(hipEventCreate(&e));
    rowwalk<V><<<grid, 64 * kWaves>>>(planes[0], planes[1], planes[2], planes[3], H, W, out);
    CHECK(hipEventRecord(a));
    for (int i = 0; i < reps; ++i)
        rowwalk<V><<<grid, 64 * kWaves>>>(planes[0], planes[1], planes[2], planes[3], H, W, out);
    CHECK(hipEventRecord(e));
    CHECK(hipEventSynchronize(e));
    float ms;
    CHECK(hipEventElapsedTime(&ms, a, e));
    return ms / reps;
}

int main() {
    const int B = 25, H = 2176, W = 4096, reps = 10;
    const size_t n = (size_t)B * H * W;
    float* planes[4];
    for (int l = 0; l < 4; ++l) {
        CHECK(hipMalloc(&planes[l], n * sizeof(float)));
        CHECK(hipMemset(planes[l], 0, n * sizeof(float)));
    }
    float* out;
    CHECK(hipMalloc(&out, n * sizeof(float)));
    const double bytes = 4.0 * n * sizeof(float) * (kStrip + 2) / kStrip;
    const float t1 = run<1>(planes, B, H, W, out, reps);
    const float t2 = run<2>(planes, B, H, W, out, reps);
    const float t4 = run<4>(planes, B, H, W, out, reps);
    printf("4-plane row walk, %d x %d x %d, %.2f GB per pass\n", B, H, W, bytes / 1e9);
    printf("dword   (64 col/wave):  %.3f ms  %.2f TB/s\n", t1, bytes / t1 / 1e9);
    printf("dwordx2 (128 col/wave): %.3f ms  %.2f TB/s\n", t2, bytes / t2 / 1e9);
    printf("dwordx4 (256 col/wave): %.3f ms  %.2f TB/s\n", t4, bytes / t4 / 1e9);
    return 0;
}
