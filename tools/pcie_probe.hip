// pcie_probe.hip -- host link rates on the GPU box, for the end-to-end numbers in DESIGN.md §5:
// DMA copies between pinned host memory and HBM (1..4 streams, each direction and both at once) and
// kernel loads / stores straight to mapped pinned host memory (16-byte vector accesses).
//   hipcc -O2 --offload-arch=gfx950 tools/pcie_probe.hip -o tools/pcie_probe && tools/pcie_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x)                                                                          \
    do {                                                                               \
        hipError_t e_ = (x);                                                           \
        if (e_ != hipSuccess) {                                                        \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                   \
        }                                                                              \
    } while (0)

__global__ void store_host(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

static double now_ms(hipEvent_t a, hipEvent_t b) {
    float ms = 0;
    CK(hipEventElapsedTime(&ms, a, b));
    return ms;
}

int main() {
    const size_t big = 512ull << 20, mid = 64ull << 20;
    void *h_a, *h_b, *d_a, *d_b;
    CK(hipHostMalloc(&h_a, big, hipHostMallocDefault));
    CK(hipHostMalloc(&h_b, big, hipHostMallocMapped));
    CK(hipMalloc(&d_a, big));
    CK(hipMalloc(&d_b, big));
    memset(h_a, 1, big);
    memset(h_b, 2, big);
    CK(hipMemset(d_a, 3, big));
    CK(hipMemset(d_b, 4, big));
    hipStream_t s[4];
    for (int k = 0; k < 4; k++) CK(hipStreamCreateWithFlags(&s[k], hipStreamNonBlocking));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    auto copy = [&](const char* what, size_t bytes, int ns, hipMemcpyKind kind, bool both) {
        double best = 1e30;
        for (int rep = 0; rep < 5; rep++) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(t0, s[0]));
            for (int k = 1; k < 4; k++) CK(hipStreamWaitEvent(s[k], t0, 0));
            const size_t piece = bytes / ns;
            for (int k = 0; k < ns; k++) {
                const size_t off = k * piece;
                if (kind == hipMemcpyHostToDevice || both)
                    CK(hipMemcpyAsync((char*)d_a + off, (char*)h_a + off, piece, hipMemcpyHostToDevice, s[k]));
                if (kind == hipMemcpyDeviceToHost || both)
                    CK(hipMemcpyAsync((char*)h_b + off, (char*)d_b + off, piece, hipMemcpyDeviceToHost,
                                      both ? s[(k + 2) & 3] : s[k]));
            }
            hipEvent_t done[4];
            for (int k = 0; k < 4; k++) {
                CK(hipEventCreateWithFlags(&done[k], hipEventDisableTiming));
                CK(hipEventRecord(done[k], s[k]));
                CK(hipStreamWaitEvent(s[0], done[k], 0));
            }
            CK(hipEventRecord(t1, s[0]));
            CK(hipEventSynchronize(t1));
            for (int k = 0; k < 4; k++) CK(hipEventDestroy(done[k]));
            const double ms = now_ms(t0, t1);
            if (ms < best) best = ms;
        }
        const double gb = (both ? 2.0 : 1.0) * bytes / 1e9;
        printf("%-34s %4zu MB x%d streams: %7.3f ms  %6.1f GB/s\n", what, bytes >> 20, ns, best, gb / (best * 1e-3));
    };
    for (size_t bytes : {mid, big})
        for (int ns : {1, 2, 4}) copy("H2D dma", bytes, ns, hipMemcpyHostToDevice, false);
    for (size_t bytes : {mid, big})
        for (int ns : {1, 2, 4}) copy("D2H dma", bytes, ns, hipMemcpyDeviceToHost, false);
    for (int ns : {1, 2}) copy("H2D + D2H dma at once (sum)", big, ns, hipMemcpyHostToDevice, true);
    // kernel stores into mapped pinned host memory, and kernel loads from it
    void* h_dev;
    CK(hipHostGetDevicePointer(&h_dev, h_b, 0));
    for (int dir = 0; dir < 2; dir++)
        for (int grid : {256, 1024, 4096}) {
            double best = 1e30;
            for (int rep = 0; rep < 5; rep++) {
                CK(hipDeviceSynchronize());
                CK(hipEventRecord(t0, s[0]));
                if (dir == 0)
                    store_host<<<grid, 256, 0, s[0]>>>((uint4*)h_dev, (const uint4*)d_b, big / 16);
                else
                    store_host<<<grid, 256, 0, s[0]>>>((uint4*)d_a, (const uint4*)h_dev, big / 16);
                CK(hipGetLastError());
                CK(hipEventRecord(t1, s[0]));
                CK(hipEventSynchronize(t1));
                const double ms = now_ms(t0, t1);
                if (ms < best) best = ms;
            }
            printf("%-34s %4zu MB grid %5d: %7.3f ms  %6.1f GB/s\n", dir == 0 ? "kernel stores to host" : "kernel loads from host",
                   big >> 20, grid, best, big / 1e9 / (best * 1e-3));
        }
    CK(hipDeviceSynchronize());
    printf("check %d %d\n", ((unsigned char*)h_b)[big - 1], ((unsigned char*)h_a)[0]);
    return 0;
}
