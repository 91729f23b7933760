// Do the first H2D copies of a process stall? 8 threads, each its own stream,
// copy 8.3 MB frames from one pinned pool to their own device buffers and sync,
// timing every hipMemcpyAsync call (host side) and every copy (event).
// usage: h2d_stall [threads] [frames] [warm_rounds] [pool_frames] [kernels 0/1]
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <thread>
#include <vector>

__global__ void touch(uint8_t* d, int n) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[(size_t)i * 4096] += 1;
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); exit(1); } } while (0)

int main(int argc, char** argv) {
    const int T = argc > 1 ? atoi(argv[1]) : 8, F = argc > 2 ? atoi(argv[2]) : 30;
    const int warm = argc > 3 ? atoi(argv[3]) : 0, P = argc > 4 ? atoi(argv[4]) : 16;
    const int kern = argc > 5 ? atoi(argv[5]) : 0;
    const size_t bytes = 1920ull * 1080 * 4;
    CK(hipSetDevice(0));
    uint8_t* pool = nullptr;
    CK(hipHostMalloc((void**)&pool, bytes * P, hipHostMallocDefault));
    for (size_t i = 0; i < bytes * P; i += 4096) pool[i] = (uint8_t)i;
    std::vector<void*> dev(2 * T);
    for (auto& d : dev) CK(hipMalloc(&d, bytes));
    std::vector<hipStream_t> st(T);
    for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    std::vector<hipEvent_t> evs(T), evn(T), evc(T);
    std::vector<hipStream_t> cst(T);
    for (auto& s2 : cst) CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    for (auto& ev2 : evc) CK(hipEventCreateWithFlags(&ev2, hipEventDisableTiming));
    for (auto& ev0 : evs) CK(hipEventCreate(&ev0));
    for (auto& ev1 : evn) CK(hipEventCreateWithFlags(&ev1, hipEventDisableTiming));
    // warm-up: `warm` rounds of copy + kernels from T threads, on the timed streams or
    // (bit 32) on streams of their own that are destroyed afterwards
    {
        std::vector<hipStream_t> ws(T);
        for (int i = 0; i < T; i++) {
            if (kern & 32) CK(hipStreamCreateWithFlags(&ws[i], hipStreamNonBlocking));
            else ws[i] = st[i];
        }
        std::vector<std::thread> wt;
        for (int i = 0; i < T; i++)
            wt.emplace_back([&, i] {
                for (int r = 0; r < warm; r++) {
                    CK(hipMemcpyAsync(dev[2 * i + (r & 1)], pool + bytes * ((r + i) % P), bytes, hipMemcpyHostToDevice, ws[i]));
                    for (int k = 0; k < 12; k++)
                        hipLaunchKernelGGL(touch, dim3(8), dim3(256), 0, ws[i], (uint8_t*)dev[2 * i + (r & 1)], 2000);
                    CK(hipStreamSynchronize(ws[i]));
                }
            });
        for (auto& t : wt) t.join();
        if (kern & 32)
            for (auto& x : ws) CK(hipStreamDestroy(x));
    }
    std::vector<std::vector<double>> api(T, std::vector<double>(F)), tot(T, std::vector<double>(F));
    using clk = std::chrono::steady_clock;
    auto t0 = clk::now();
    std::vector<std::thread> th;
    for (int i = 0; i < T; i++)
        th.emplace_back([&, i] {
            for (int f = 0; f < F; f++) {
                auto a = clk::now();
                // bit 16: the copy on its own stream (no kernels ever on it), the kernel stream waits on an event
                hipStream_t cs_ = (kern & 16) ? cst[i] : st[i];
                CK(hipMemcpyAsync(dev[2 * i + (f & 1)], pool + bytes * ((f + 3 * i) % P), bytes, hipMemcpyHostToDevice, cs_));
                if (kern & 16) {
                    CK(hipEventRecord(evc[i], cs_));
                    CK(hipStreamWaitEvent(st[i], evc[i], 0));
                }
                auto b = clk::now();
                // kern bits: 1 kernels behind the copy, 2 record+sync a persistent event,
                // 4 create/destroy an event per frame, 8 timing-disabled persistent event
                if (kern & 1)
                    for (int k = 0; k < 12; k++)
                        hipLaunchKernelGGL(touch, dim3(8), dim3(256), 0, st[i], (uint8_t*)dev[2 * i + (f & 1)], 2000);
                if (kern & 2) {
                    CK(hipEventRecord(evs[i], st[i]));
                    CK(hipEventSynchronize(evs[i]));
                }
                if (kern & 8) {
                    CK(hipEventRecord(evn[i], st[i]));
                    CK(hipEventSynchronize(evn[i]));
                }
                if (kern & 4) {
                    hipEvent_t ev;
                    CK(hipEventCreate(&ev));
                    CK(hipEventRecord(ev, st[i]));
                    CK(hipEventSynchronize(ev));
                    CK(hipEventDestroy(ev));
                }
                CK(hipStreamSynchronize(st[i]));
                auto c = clk::now();
                api[i][f] = std::chrono::duration<double, std::milli>(b - a).count();
                tot[i][f] = std::chrono::duration<double, std::milli>(c - a).count();
            }
        });
    for (auto& t : th) t.join();
    double el = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    int stalls = 0;
    for (int f = 0; f < F; f++)
        for (int i = 0; i < T; i++) stalls += f > 0 && api[i][f] > 2.0;
    printf("threads %d frames %d warm %d pool %d kern %d: %.1f ms total, %.2f GB/s, stalled calls after frame 0: %d\n", T, F, warm, P, kern, el,
           T * F * bytes / el / 1e6, stalls);
    for (int f = 0; f < F && getenv("VERBOSE"); f++) {
        double mx = 0, mt = 0;
        for (int i = 0; i < T; i++) { mx = std::max(mx, api[i][f]); mt = std::max(mt, tot[i][f]); }
        printf("frame %2d: max api %.2f ms, max api+sync %.2f ms\n", f, mx, mt);
    }
    return 0;
}
