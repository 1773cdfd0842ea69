// PCIe probe for the host-buffer path (tools/pcie_bench.hip; build: hipcc --offload-arch=gfx950 -O2
// tools/pcie_bench.hip -o tools/pcie_bench).  Sizes are one 2048-stream ByteTrack step: 100 MB
// of detections in, 134 MB of output rows out.  Measures, over REP repetitions each:
//   sdma_h2d / sdma_d2h      hipMemcpyAsync alone (copy engines)
//   sdma_duplex              both at once on two streams
//   kern_d2h_<blocks>        a kernel storing device rows straight into mapped host memory
//   kern_h2d_<blocks>        a kernel loading mapped host memory into device memory
//   duplex_sdma_in_kern_out  copy-engine H2D beside a kernel D2H
// and prints one JSON object, plus the process's CPU list and the GPU's NUMA node.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <vector>

#define CK(x)                                                                              \
    do {                                                                                   \
        hipError_t e_ = (x);                                                               \
        if (e_ != hipSuccess) {                                                            \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                       \
        }                                                                                  \
    } while (0)

// grid-stride 16-B copy; src / dst may be mapped host memory
__global__ void k_copy16(const uint4 *__restrict__ src, uint4 *__restrict__ dst, size_t n) {
    const size_t stride = (size_t)gridDim.x * blockDim.x;
    for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride)
        dst[i] = src[i];
}

static double now_ms() {
    return std::chrono::duration<double, std::milli>(
               std::chrono::steady_clock::now().time_since_epoch())
        .count();
}

static std::string slurp(const char *p) {
    std::ifstream f(p);
    std::string s, line;
    while (std::getline(f, line)) s += line;
    return s;
}

int main(int argc, char **argv) {
    const size_t H2D = 100663296, D2H = 134217728;
    const int REP = argc > 1 ? atoi(argv[1]) : 10;
    CK(hipSetDevice(0));
    void *hin, *hout, *din, *dout;
    CK(hipHostMalloc(&hin, H2D, hipHostMallocDefault));
    CK(hipHostMalloc(&hout, D2H, hipHostMallocDefault));
    CK(hipMalloc(&din, H2D));
    CK(hipMalloc(&dout, D2H));
    memset(hin, 1, H2D);
    memset(hout, 2, D2H);
    CK(hipMemset(din, 3, H2D));
    CK(hipMemset(dout, 4, D2H));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    void *hin_d = nullptr, *hout_d = nullptr;
    CK(hipHostGetDevicePointer(&hin_d, hin, 0));
    CK(hipHostGetDevicePointer(&hout_d, hout, 0));

    auto timed = [&](auto fn) {
        fn();
        CK(hipDeviceSynchronize());
        const double t0 = now_ms();
        for (int r = 0; r < REP; ++r) fn();
        CK(hipDeviceSynchronize());
        return (now_ms() - t0) / REP;
    };
    auto h2d = [&] { CK(hipMemcpyAsync(din, hin, H2D, hipMemcpyHostToDevice, s1)); };
    auto d2h = [&] { CK(hipMemcpyAsync(hout, dout, D2H, hipMemcpyDeviceToHost, s2)); };
    auto kd2h = [&](int blocks) {
        hipLaunchKernelGGL(k_copy16, dim3(blocks), dim3(256), 0, s2, (const uint4 *)dout,
                           (uint4 *)hout_d, D2H / 16);
    };
    auto kh2d = [&](int blocks) {
        hipLaunchKernelGGL(k_copy16, dim3(blocks), dim3(256), 0, s1, (const uint4 *)hin_d,
                           (uint4 *)din, H2D / 16);
    };
    std::string js = "{";
    auto put = [&](const char *k, double ms, size_t bytes) {
        char b[160];
        snprintf(b, sizeof b, "%s\"%s\": {\"ms\": %.4f, \"gbs\": %.2f}", js.size() > 1 ? ", " : "",
                 k, ms, bytes / ms / 1e6);
        js += b;
    };
    for (int rep = 0; rep < 2; ++rep) {   // twice: run-to-run variation inside one process
        const std::string sfx = rep ? "_again" : "";
        put(("sdma_h2d" + sfx).c_str(), timed(h2d), H2D);
        put(("sdma_d2h" + sfx).c_str(), timed(d2h), D2H);
        put(("sdma_duplex" + sfx).c_str(), timed([&] { h2d(); d2h(); }), H2D + D2H);
    }
    for (int blocks : {64, 256, 1024, 4096}) {
        char k[64];
        snprintf(k, sizeof k, "kern_d2h_%d", blocks);
        put(k, timed([&] { kd2h(blocks); }), D2H);
        snprintf(k, sizeof k, "kern_h2d_%d", blocks);
        put(k, timed([&] { kh2d(blocks); }), H2D);
    }
    put("duplex_sdma_in_kern_out_1024", timed([&] { h2d(); kd2h(1024); }), H2D + D2H);
    put("duplex_kern_out_then_sdma_in_128", timed([&] { kd2h(128); h2d(); }), H2D + D2H);
    put("duplex_sdma_in_then_kern_out_128", timed([&] { h2d(); kd2h(128); }), H2D + D2H);
    {   // when does a copy-engine H2D start if a kernel D2H is already streaming?
        hipEvent_t e0, e1, e2, e3;
        for (hipEvent_t *ev : {&e0, &e1, &e2, &e3}) CK(hipEventCreate(ev));
        float a = 0, b = 0, c = 0;
        double sa = 0, sb = 0, sc = 0;
        for (int r = 0; r < REP; ++r) {
            CK(hipDeviceSynchronize());
            CK(hipEventRecord(e0, s2));
            kd2h(128);
            CK(hipEventRecord(e1, s2));
            CK(hipEventRecord(e2, s1));
            h2d();
            CK(hipEventRecord(e3, s1));
            CK(hipDeviceSynchronize());
            CK(hipEventElapsedTime(&a, e0, e1));   // kernel D2H
            CK(hipEventElapsedTime(&b, e0, e2));   // H2D start after the kernel's start
            CK(hipEventElapsedTime(&c, e2, e3));   // H2D duration
            sa += a; sb += b; sc += c;
        }
        char buf[200];
        snprintf(buf, sizeof buf, ", \"overlap_probe\": {\"kern_d2h_ms\": %.3f, \"h2d_start_after_ms\": %.3f, \"h2d_ms\": %.3f}",
                 sa / REP, sb / REP, sc / REP);
        js += buf;
    }
    put("duplex_kern_in_sdma_out_1024", timed([&] { kh2d(1024); d2h(); }), H2D + D2H);
    put("duplex_kern_both_1024", timed([&] { kh2d(1024); kd2h(1024); }), H2D + D2H);
    int node = -1;
    {
        char bus[64] = {0};
        CK(hipDeviceGetPCIBusId(bus, sizeof bus, 0));
        for (char *c = bus; *c; ++c) *c = (char)tolower(*c);
        std::string p = std::string("/sys/bus/pci/devices/") + bus + "/numa_node";
        std::string v = slurp(p.c_str());
        if (!v.empty()) node = atoi(v.c_str());
        js += std::string(", \"pci_bus\": \"") + bus + "\"";
    }
    std::string cpus;
    {
        std::ifstream f("/proc/self/status");
        std::string line;
        while (std::getline(f, line))
            if (line.rfind("Cpus_allowed_list", 0) == 0) cpus = line.substr(line.find(':') + 1);
    }
    while (!cpus.empty() && (cpus[0] == ' ' || cpus[0] == '\t')) cpus.erase(0, 1);
    char tail[512];
    snprintf(tail, sizeof tail, ", \"gpu_numa_node\": %d, \"cpus_allowed\": \"%s\", \"nodes\": \"%s\"}",
             node, cpus.c_str(), slurp("/sys/devices/system/node/online").c_str());
    js += tail;
    printf("%s\n", js.c_str());
    return 0;
}
