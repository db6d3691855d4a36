// Host-side launch cost on this box: empty kernels, back-to-back launches,
// a captured 4-kernel graph, and small D2H readback round trips.
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_empty(int *p) {
    if (p && threadIdx.x == 0 && blockIdx.x == 0) p[0] += 1;
}

static double now_us() {
    return std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

__global__ void k_publish(volatile long long *host, long long seq) {
    if (threadIdx.x == 0 && blockIdx.x == 0) {
        __threadfence_system();
        host[0] = seq;
    }
}

int main(int argc, char **argv) {
    if (argc > 1 && argv[1][0] == 's') {
        printf("hipSetDeviceFlags(spin) -> %d\n", (int)hipSetDeviceFlags(hipDeviceScheduleSpin));
    }
    if (argc > 1 && argv[1][0] == 'y') {
        printf("hipSetDeviceFlags(yield) -> %d\n", (int)hipSetDeviceFlags(hipDeviceScheduleYield));
    }
    hipStream_t s;
    hipStreamCreateWithFlags(&s, hipStreamNonBlocking);
    int *d;
    hipMalloc(&d, 64);
    long long *pin;
    hipHostMalloc(&pin, 64, hipHostMallocDefault);
    for (int i = 0; i < 100; i++) hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, d);
    hipStreamSynchronize(s);
    const int N = 2000;
    double t0 = now_us();
    for (int i = 0; i < N; i++) hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, d);
    double t1 = now_us();
    hipStreamSynchronize(s);
    double t2 = now_us();
    printf("launch: host %.2f us/launch, total incl drain %.2f us/launch\n", (t1 - t0) / N, (t2 - t0) / N);
    // launch + 8-byte D2H + sync round trip
    t0 = now_us();
    for (int i = 0; i < 200; i++) {
        hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, d);
        hipMemcpyAsync(pin, d, 8, hipMemcpyDeviceToHost, s);
        hipStreamSynchronize(s);
    }
    t1 = now_us();
    printf("launch+d2h8+sync round trip: %.2f us\n", (t1 - t0) / 200);
    // same with spin on hipStreamQuery
    t0 = now_us();
    for (int i = 0; i < 200; i++) {
        hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, d);
        hipMemcpyAsync(pin, d, 8, hipMemcpyDeviceToHost, s);
        while (hipStreamQuery(s) == hipErrorNotReady) {
        }
    }
    t1 = now_us();
    printf("launch+d2h8+spin query round trip: %.2f us\n", (t1 - t0) / 200);
    // graph of 4 kernels
    hipGraph_t g;
    hipGraphExec_t ge;
    hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
    for (int i = 0; i < 4; i++) hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, d);
    hipStreamEndCapture(s, &g);
    hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
    hipGraphLaunch(ge, s);
    hipStreamSynchronize(s);
    t0 = now_us();
    for (int i = 0; i < 500; i++) hipGraphLaunch(ge, s);
    t1 = now_us();
    hipStreamSynchronize(s);
    t2 = now_us();
    printf("graph(4 kernels): host %.2f us/launch, incl drain %.2f us/launch\n", (t1 - t0) / 500, (t2 - t0) / 500);
    // 4 separate launches + sync round trip vs graph + sync
    t0 = now_us();
    for (int i = 0; i < 200; i++) {
        for (int k = 0; k < 4; k++) hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, d);
        hipStreamSynchronize(s);
    }
    t1 = now_us();
    printf("4 launches + sync: %.2f us\n", (t1 - t0) / 200);
    t0 = now_us();
    for (int i = 0; i < 200; i++) {
        hipGraphLaunch(ge, s);
        hipStreamSynchronize(s);
    }
    t1 = now_us();
    printf("graph + sync: %.2f us\n", (t1 - t0) / 200);
    t0 = now_us();
    for (int i = 0; i < 200; i++) {
        hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, d);
        hipStreamSynchronize(s);
    }
    t1 = now_us();
    printf("1 launch + sync: %.2f us\n", (t1 - t0) / 200);
    // kernel publishes a sequence number into pinned host memory; host spins on it
    volatile long long *mb;
    hipHostMalloc((void **)&mb, 64, hipHostMallocCoherent | hipHostMallocMapped);
    mb[0] = 0;
    t0 = now_us();
    for (int i = 1; i <= 500; i++) {
        hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, d);
        hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, s, mb, (long long)i);
        while (mb[0] != i) {
        }
    }
    t1 = now_us();
    printf("launch+publish+spin round trip: %.2f us\n", (t1 - t0) / 500);
    t0 = now_us();
    for (int i = 501; i <= 1000; i++) {
        hipLaunchKernelGGL(k_publish, dim3(1), dim3(64), 0, s, mb, (long long)i);
        while (mb[0] != i) {
        }
    }
    t1 = now_us();
    printf("publish-only+spin round trip: %.2f us\n", (t1 - t0) / 500);
    hipStreamSynchronize(s);
    // event-based wait
    hipEvent_t ev;
    hipEventCreateWithFlags(&ev, hipEventDisableTiming);
    t0 = now_us();
    for (int i = 0; i < 200; i++) {
        hipLaunchKernelGGL(k_empty, dim3(1024), dim3(256), 0, s, d);
        hipEventRecord(ev, s);
        hipEventSynchronize(ev);
    }
    t1 = now_us();
    printf("launch+event sync: %.2f us\n", (t1 - t0) / 200);
    return 0;
}
