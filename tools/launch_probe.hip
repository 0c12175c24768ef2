/* launch cost of a kernel that follows a busy kernel on the same stream, by
 * the follower's resources (empty body: it reads a zero count and returns):
 *   light / 145 KiB LDS / 48 B scratch / both (the list-mode lane kernel's shape)
 * build: hipcc --offload-arch=gfx950 -O3 -o tools/launch_probe tools/launch_probe.hip */
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define CHK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ __launch_bounds__(256) void busy(uint32_t *out, uint32_t n)
{
    __shared__ uint32_t s[9000];
    uint32_t v = threadIdx.x;
    for (uint32_t k = 0; k < n; k++) {
        s[(threadIdx.x * 7 + k) % 9000] = v;
        __syncthreads();
        v = v * 1664525u + s[(threadIdx.x * 13 + k) % 9000];
    }
    out[blockIdx.x * 256 + threadIdx.x] = v;
}
__global__ __launch_bounds__(256) void f_light(const uint32_t *cnt, uint32_t *out)
{
    if (*cnt == 0) return;
    out[threadIdx.x] = 1;
}
__global__ __launch_bounds__(256) void f_lds(const uint32_t *cnt, uint32_t *out)
{
    __shared__ uint64_t big[145 * 1024 / 8];
    if (*cnt == 0) return;
    big[threadIdx.x] = threadIdx.x;
    __syncthreads();
    out[threadIdx.x] = (uint32_t)big[(threadIdx.x * 5) % 256];
}
__device__ __noinline__ uint32_t deep(volatile uint32_t *a, uint32_t i)
{
    a[i % 12] = i;
    return a[(i * 7) % 12];
}
__global__ __launch_bounds__(256) void f_scratch(const uint32_t *cnt, uint32_t *out)
{
    volatile uint32_t arr[12];
    if (*cnt == 0) return;
    out[threadIdx.x] = deep(arr, threadIdx.x);
}
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void f_both(const uint32_t *cnt, uint32_t *out)
{
    __shared__ uint64_t big[145 * 1024 / 8];
    volatile uint32_t arr[12];
    if (*cnt == 0) return;
    big[threadIdx.x] = deep(arr, threadIdx.x);
    __syncthreads();
    out[threadIdx.x] = (uint32_t)big[(threadIdx.x * 5) % 256];
}

int main()
{
    uint32_t *cnt, *out;
    CHK(hipMalloc(&cnt, 4));
    CHK(hipMemset(cnt, 0, 4));
    CHK(hipMalloc(&out, 1024 * 256 * 4));
    hipStream_t s;
    CHK(hipStreamCreate(&s));
    hipEvent_t e0, e1;
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const int iters = 300;
    const char *names[] = {"busy only", "busy + light", "busy + 145KiB LDS", "busy + 48B scratch", "busy + both"};
    for (int rep = 0; rep < 2; rep++)
        for (int v = 0; v < 5; v++) {
            CHK(hipEventRecord(e0, s));
            for (int i = 0; i < iters; i++) {
                hipLaunchKernelGGL(busy, dim3(1024), dim3(256), 0, s, out, 64u);
                if (v == 1) hipLaunchKernelGGL(f_light, dim3(16), dim3(256), 0, s, cnt, out);
                if (v == 2) hipLaunchKernelGGL(f_lds, dim3(16), dim3(256), 0, s, cnt, out);
                if (v == 3) hipLaunchKernelGGL(f_scratch, dim3(16), dim3(256), 0, s, cnt, out);
                if (v == 4) hipLaunchKernelGGL(f_both, dim3(16), dim3(256), 0, s, cnt, out);
            }
            CHK(hipGetLastError());
            CHK(hipEventRecord(e1, s));
            CHK(hipEventSynchronize(e1));
            float ms = 0;
            CHK(hipEventElapsedTime(&ms, e0, e1));
            if (rep) printf("%-22s %8.2f us per iteration\n", names[v], ms * 1000 / iters);
        }
    return 0;
}
