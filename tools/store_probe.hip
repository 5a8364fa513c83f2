// store_probe.hip -- shader stores into pinned host memory by allocation flags (default, mapped,
// coherent, non-coherent) and size, plus the copy engine's DMA into the same memory: which pinned
// memory the engine's arenas (mxp_host_alloc) should be.
//   hipcc -O2 --offload-arch=gfx950 tools/store_probe.hip -o tools/store_probe && tools/store_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

__global__ void copy16(uint4* __restrict__ dst, const uint4* __restrict__ src, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        dst[i] = src[i];
}

int main() {
    const size_t big = 768ull << 20;
    void* d;
    CK(hipMalloc(&d, big));
    CK(hipMemset(d, 5, big));
    hipEvent_t t0, t1;
    CK(hipEventCreate(&t0));
    CK(hipEventCreate(&t1));
    struct F {
        const char* name;
        unsigned flags;
    } fl[] = {{"default", hipHostMallocDefault},
              {"mapped", hipHostMallocMapped},
              {"coherent", hipHostMallocCoherent},
              {"noncoherent", hipHostMallocNonCoherent},
              {"mapped|noncoherent", hipHostMallocMapped | hipHostMallocNonCoherent},
              {"portable", hipHostMallocPortable}};
    for (const F& f : fl) {
        void* h;
        if (hipHostMalloc(&h, big, f.flags) != hipSuccess) {
            printf("%-20s alloc failed\n", f.name);
            (void)hipGetLastError();
            continue;
        }
        memset(h, 0, big);
        void* hd = nullptr;
        CK(hipHostGetDevicePointer(&hd, h, 0));
        for (size_t bytes : {(size_t)64 << 20, big}) {
            double best_k = 1e30, best_d = 1e30;
            for (int rep = 0; rep < 4; rep++) {
                CK(hipEventRecord(t0, 0));
                copy16<<<1024, 256>>>((uint4*)hd, (const uint4*)d, bytes / 16);
                CK(hipEventRecord(t1, 0));
                CK(hipEventSynchronize(t1));
                float ms;
                CK(hipEventElapsedTime(&ms, t0, t1));
                if (ms < best_k) best_k = ms;
                CK(hipEventRecord(t0, 0));
                CK(hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, 0));
                CK(hipEventRecord(t1, 0));
                CK(hipEventSynchronize(t1));
                CK(hipEventElapsedTime(&ms, t0, t1));
                if (ms < best_d) best_d = ms;
            }
            printf("%-20s %4zu MB: shader %6.1f GB/s  dma %6.1f GB/s  (check %d)\n", f.name, bytes >> 20,
                   bytes / 1e9 / (best_k * 1e-3), bytes / 1e9 / (best_d * 1e-3), ((unsigned char*)h)[bytes - 1]);
        }
        CK(hipHostFree(h));
    }
    return 0;
}
