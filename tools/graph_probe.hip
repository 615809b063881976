// graph_probe.hip — host cost per frame of 6 dependent small kernels: direct hipLaunchKernel with
// a 1.2 KiB / 64 B argument vs one hipGraphLaunch of the captured frame (with one kernel-node
// parameter update per frame, as a changing depth pointer would need).
#include <hip/hip_runtime.h>
#include <chrono>
#include <stdio.h>
#include <vector>
#pragma clang diagnostic ignored "-Wunused-value"
#pragma clang diagnostic ignored "-Wunused-result"

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("%s line %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

struct BigArgs { float v[296]; int* p; int* q; };
struct SmallArgs { float v[12]; int* p; int* q; };

template <class A>
__global__ void k_work(A a) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    a.q[i] = a.p[i] + (int)a.v[threadIdx.x & 7];
}

using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::micro>(b - a).count(); }

template <class F>
void run(const char* name, hipStream_t s, F frame) {
    for (int i = 0; i < 100; ++i) frame(i);
    hipStreamSynchronize(s);
    double host = 0;
    const int n = 3000;
    auto t0 = clk::now();
    for (int i = 0; i < n; ++i) {
        if (i % 16 == 0) {  // drain outside the host timer so the queue never fills
            hipStreamSynchronize(s);
        }
        auto a = clk::now();
        frame(i);
        host += us(a, clk::now());
    }
    hipStreamSynchronize(s);
    auto t1 = clk::now();
    // steady-state throughput without drains
    auto t2 = clk::now();
    for (int i = 0; i < n; ++i) frame(i);
    hipStreamSynchronize(s);
    auto t3 = clk::now();
    printf("%-34s host %6.2f us/frame   throughput %6.2f us/frame\n", name, host / n, us(t2, t3) / n);
    (void)t0; (void)t1;
}

int main() {
    hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    int *p, *q; CK(hipMalloc(&p, 1 << 22)); CK(hipMalloc(&q, 1 << 22));
    CK(hipMemset(p, 0, 1 << 22)); CK(hipMemset(q, 0, 1 << 22));
    BigArgs big{}; big.p = p; big.q = q;
    SmallArgs sm{}; sm.p = p; sm.q = q;
    const dim3 grid(300), block(256);
    run("direct 6x big (1.2 KiB) args", s, [&](int i) {
        big.v[0] = (float)i;
        for (int k = 0; k < 6; ++k) hipLaunchKernelGGL(k_work<BigArgs>, grid, block, 0, s, big);
    });
    run("direct 6x small (64 B) args", s, [&](int i) {
        sm.v[0] = (float)i;
        for (int k = 0; k < 6; ++k) hipLaunchKernelGGL(k_work<SmallArgs>, grid, block, 0, s, sm);
    });
    run("direct 4x big args", s, [&](int i) {
        big.v[0] = (float)i;
        for (int k = 0; k < 4; ++k) hipLaunchKernelGGL(k_work<BigArgs>, grid, block, 0, s, big);
    });
    // graph of the 6-kernel frame
    hipGraph_t g; hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < 6; ++k) hipLaunchKernelGGL(k_work<BigArgs>, grid, block, 0, s, big);
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    size_t nn = 0; CK(hipGraphGetNodes(g, nullptr, &nn));
    std::vector<hipGraphNode_t> nodes(nn); CK(hipGraphGetNodes(g, nodes.data(), &nn));
    run("graph 6x big, no update", s, [&](int) { hipGraphLaunch(ge, s); });
    run("graph 6x big, 1 node update", s, [&](int i) {
        big.v[0] = (float)i;
        void* args[] = {&big};
        hipKernelNodeParams kp{};
        kp.func = (void*)k_work<BigArgs>;
        kp.gridDim = grid; kp.blockDim = block; kp.sharedMemBytes = 0;
        kp.kernelParams = args; kp.extra = nullptr;
        hipGraphExecKernelNodeSetParams(ge, nodes[0], &kp);
        hipGraphLaunch(ge, s);
    });
    // per frame: re-capture the frame, whole-graph update of the executable, launch
    run("capture + exec update + launch", s, [&](int i) {
        big.v[0] = (float)i;
        hipGraph_t g2;
        hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int k = 0; k < 6; ++k) hipLaunchKernelGGL(k_work<BigArgs>, grid, block, 0, s, big);
        hipStreamEndCapture(s, &g2);
        hipGraphNode_t en;
        hipGraphExecUpdateResult ur;
        if (hipGraphExecUpdate(ge, g2, &en, &ur) != hipSuccess) printf("update failed\n");
        hipGraphLaunch(ge, s);
        hipGraphDestroy(g2);
    });
    run("graph 6x big, 6 node updates", s, [&](int i) {
        big.v[0] = (float)i;
        void* args[] = {&big};
        hipKernelNodeParams kp{};
        kp.func = (void*)k_work<BigArgs>;
        kp.gridDim = grid; kp.blockDim = block; kp.sharedMemBytes = 0;
        kp.kernelParams = args; kp.extra = nullptr;
        for (int k = 0; k < 6; ++k) hipGraphExecKernelNodeSetParams(ge, nodes[k], &kp);
        hipGraphLaunch(ge, s);
    });
    // three small graphs per frame (2 + 1 + 3 kernels) with an event record in between
    hipGraph_t ga, gb, gc; hipGraphExec_t ea, eb, ec;
    hipEvent_t ev; CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    auto cap = [&](int m, hipGraph_t* gg, hipGraphExec_t* ee) {
        hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal);
        for (int k = 0; k < m; ++k) hipLaunchKernelGGL(k_work<BigArgs>, grid, block, 0, s, big);
        hipStreamEndCapture(s, gg);
        hipGraphInstantiate(ee, *gg, nullptr, nullptr, 0);
    };
    cap(2, &ga, &ea); cap(1, &gb, &eb); cap(3, &gc, &ec);
    run("3 graphs + event record + wait", s, [&](int) {
        hipGraphLaunch(ea, s);
        hipStreamWaitEvent(s, ev, 0);
        hipGraphLaunch(eb, s);
        hipEventRecord(ev, s);
        hipGraphLaunch(ec, s);
    });
    run("graph + event record", s, [&](int) {
        hipGraphLaunch(ge, s);
        hipEventRecord(ev, s);
    });
    // two streams alternating frames (graph per stream), with / without an event chain
    hipStream_t s2; CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipGraphExec_t ge2;
    CK(hipGraphInstantiate(&ge2, g, nullptr, nullptr, 0));
    hipEvent_t e1, e2;
    CK(hipEventCreateWithFlags(&e1, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&e2, hipEventDisableTiming));
    auto run2 = [&](const char* name, bool chain, bool rec) {
        for (int rep = 0; rep < 2; ++rep) {
            const int n = 3000;
            auto a = clk::now();
            for (int i = 0; i < n; ++i) {
                hipStream_t st = (i & 1) ? s2 : s;
                hipEvent_t mine = (i & 1) ? e2 : e1, other = (i & 1) ? e1 : e2;
                if (chain && i > 0) hipStreamWaitEvent(st, other, 0);
                hipGraphLaunch((i & 1) ? ge2 : ge, st);
                if (rec) hipEventRecord(mine, st);
            }
            hipStreamSynchronize(s);
            hipStreamSynchronize(s2);
            if (rep) printf("%-34s throughput %6.2f us/frame\n", name, us(a, clk::now()) / n);
        }
    };
    run2("2 streams, independent", false, false);
    run2("2 streams, records only", false, true);
    run2("2 streams, record + wait chain", true, true);
    return 0;
}
