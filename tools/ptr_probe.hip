// ptr_probe.hip -- what hipPointerGetAttributes reports for pinned host memory (hipHostMalloc with
// default and mapped flags) at the allocation's base and at an offset, and for pageable memory;
// then a shader copy through the reported device pointer, checked on the host.
//   hipcc -O2 --offload-arch=gfx950 tools/ptr_probe.hip -o tools/ptr_probe && tools/ptr_probe
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

__global__ void fill(uint8_t* d, uint64_t n, uint8_t v) {
    for (uint64_t i = blockIdx.x * 256ull + threadIdx.x; i < n; i += gridDim.x * 256ull) d[i] = v;
}

static void show(const char* what, const void* p) {
    hipPointerAttribute_t pa;
    memset(&pa, 0, sizeof pa);
    hipError_t e = hipPointerGetAttributes(&pa, p);
    printf("%-28s p=%p rc=%d type=%d device=%d hostPointer=%p devicePointer=%p flags=%u\n", what, p, (int)e, (int)pa.type,
           pa.device, pa.hostPointer, pa.devicePointer, pa.allocationFlags);
    (void)hipGetLastError();
}

int main() {
    void *a, *b;
    if (hipHostMalloc(&a, 1 << 20, hipHostMallocDefault) != hipSuccess) return 1;
    if (hipHostMalloc(&b, 1 << 20, hipHostMallocMapped) != hipSuccess) return 1;
    void* c = malloc(1 << 20);
    show("default base", a);
    show("default +4099", (char*)a + 4099);
    show("mapped base", b);
    show("mapped +4099", (char*)b + 4099);
    show("pageable", c);
    void* dp = nullptr;
    hipError_t e = hipHostGetDevicePointer(&dp, (char*)a + 4099, 0);
    printf("hipHostGetDevicePointer(default +4099) rc=%d -> %p\n", (int)e, dp);
    (void)hipGetLastError();
    hipPointerAttribute_t pa;
    if (hipPointerGetAttributes(&pa, (char*)a + 4099) == hipSuccess && pa.devicePointer) {
        const char* hp = (const char*)pa.hostPointer;
        uint8_t* d = (uint8_t*)pa.devicePointer + ((char*)a + 4099 - hp);
        memset(a, 0, 1 << 20);
        hipLaunchKernelGGL(fill, dim3(4), dim3(256), 0, 0, d, 1000, (uint8_t)7);
        if (hipDeviceSynchronize() != hipSuccess) return 2;
        int ok = 1;
        for (int i = 0; i < 1 << 20; i++) ok &= ((uint8_t*)a)[i] == ((i >= 4099 && i < 5099) ? 7 : 0);
        printf("shader fill through the derived pointer: %s\n", ok ? "ok" : "WRONG BYTES");
    }
    return 0;
}
