// Host -> device copy rate of a page-locked 448 MiB trace (28 columns x 16 MiB) under the conditions a proof
// creates: nothing else running; a busy kernel on another stream filling every CU; a stream parked behind a
// cross-stream event wait (barrier packet) while the copies run; the host spinning in a stream sync.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 upload_probe.hip -o upload_probe
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

__global__ void busy(uint64_t cycles, uint64_t *sink) {
    const uint64_t t0 = wall_clock64();
    uint64_t x = threadIdx.x;
    while (wall_clock64() - t0 < cycles) x = x * 6364136223846793005ull + 1442695040888963407ull;
    if (x == 42) sink[0] = x;
}

// mode 1: the copy stream first waits on an (already complete) event of another stream; mode 2: an event is
// recorded after every 7 columns (the prover's upload groups); mode 3: both
static hipStream_t g_other;
static uint32_t *g_flag;
static float copies(hipStream_t s, uint8_t *d, const uint8_t *h, size_t col, int ncol, int mode = 0) {
    hipEvent_t a, b, e1, eg[4];
    (void)hipEventCreate(&a);
    (void)hipEventCreate(&b);
    (void)hipEventCreateWithFlags(&e1, hipEventDisableTiming);
    for (auto &e : eg) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
    if (mode & 1) {
        (void)hipEventRecord(e1, g_other);
        (void)hipStreamWaitEvent(s, e1, 0);
    }
    (void)hipEventRecord(a, s);
    if (mode == 8) {  // one 112 MiB copy per group of 7 columns, an event after each
        for (int g = 0; g < 4; g++) {
            (void)hipMemcpyAsync(d + g * 7 * col, h + g * 7 * col, 7 * col, hipMemcpyHostToDevice, s);
            (void)hipEventRecord(eg[g], s);
        }
    } else {
        for (int c = 0; c < ncol; c++) {
            (void)hipMemcpyAsync(d + c * col, h + c * col, col, hipMemcpyHostToDevice, s);
            if ((mode & 2) && c % 7 == 6) (void)hipEventRecord(eg[c / 7], s);
            if ((mode & 4) && c % 7 == 6) (void)hipStreamWriteValue32(s, g_flag, (uint32_t)(c / 7 + 1), 0);
        }
    }
    (void)hipEventRecord(b, s);
    (void)hipEventSynchronize(b);
    float ms = 0;
    (void)hipEventElapsedTime(&ms, a, b);
    (void)hipEventDestroy(a);
    (void)hipEventDestroy(b);
    (void)hipEventDestroy(e1);
    for (auto &e : eg) (void)hipEventDestroy(e);
    return ms;
}

int main(int argc, char **argv) {
    if (argc > 1 && argv[1][0] == 's') CK(hipSetDeviceFlags(hipDeviceScheduleSpin));
    const size_t col = (size_t)16 << 20;
    const int ncol = 28;
    uint8_t *h, *d;
    uint64_t *sink;
    CK(hipHostMalloc((void **)&h, col * ncol, hipHostMallocPortable));
    for (size_t i = 0; i < col * ncol; i += 4096) h[i] = (uint8_t)i;
    CK(hipMalloc((void **)&d, col * ncol));
    CK(hipMalloc((void **)&sink, 8));
    hipStream_t sc, sk, sw;
    CK(hipStreamCreateWithFlags(&sc, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sk, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&sw, hipStreamNonBlocking));
    int clk_khz = 100000;
    (void)hipDeviceGetAttribute(&clk_khz, hipDeviceAttributeWallClockRate, 0);
    const uint64_t busy_cycles = (uint64_t)clk_khz * 40;  // ~40 ms
    const double gb = (double)col * ncol / 1e9;
    g_other = sk;
    CK(hipMalloc((void **)&g_flag, 64));
    for (int rep = 0; rep < 2; rep++)
        for (int mode : {0, 1, 2, 3, 4, 8}) {
            const float t = copies(sc, d, h, col, ncol, mode);
            printf("rep %d mode %d (1: after a cross-stream wait, 2: events per group, 4: write-value per group, 8: 4 big copies + events) %7.2f ms %6.1f GB/s\n", rep, mode, t,
                   gb / t * 1e3);
        }
    for (int rep = 0; rep < 3; rep++) {
        float t = copies(sc, d, h, col, ncol);
        printf("rep %d alone                         %7.2f ms %6.1f GB/s\n", rep, t, gb / t * 1e3);
        hipLaunchKernelGGL(busy, dim3(256 * 8), dim3(256), 0, sk, busy_cycles, sink);
        t = copies(sc, d, h, col, ncol);
        printf("rep %d beside a busy kernel          %7.2f ms %6.1f GB/s\n", rep, t, gb / t * 1e3);
        CK(hipStreamSynchronize(sk));
        // a stream parked on an event of a stream that is still busy: a barrier packet waits while we copy
        hipEvent_t ev;
        CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, sk, busy_cycles, sink);
        CK(hipEventRecord(ev, sk));
        CK(hipStreamWaitEvent(sw, ev, 0));
        hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, sw, 1000, sink);
        t = copies(sc, d, h, col, ncol);
        printf("rep %d beside a parked event wait    %7.2f ms %6.1f GB/s\n", rep, t, gb / t * 1e3);
        CK(hipStreamSynchronize(sw));
        CK(hipEventDestroy(ev));
        // one small kernel on another stream while the copies run
        hipLaunchKernelGGL(busy, dim3(1), dim3(64), 0, sk, busy_cycles, sink);
        t = copies(sc, d, h, col, ncol);
        printf("rep %d beside a 1-wave kernel        %7.2f ms %6.1f GB/s\n", rep, t, gb / t * 1e3);
        CK(hipStreamSynchronize(sk));
    }
    return 0;
}
