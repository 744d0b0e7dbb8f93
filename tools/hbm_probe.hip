// hbm_probe.hip -- practical HBM ceilings of one MI355X for the fused modem kernels' access
// pattern: streaming loads / stores over a buffer the size of one bench launch (1e6 OFDM
// symbols x 1024 complex64 = 8.19 GB), 512-thread workgroups.
//
//   hipcc --offload-arch=gfx950 -O3 tools/hbm_probe.hip -o tools/hbm_probe && tools/hbm_probe
//
// Prints one JSON line, GB/s per variant:
//   read/write  x  {16-byte lanes (dwordx4), 8-byte lanes (dwordx2, one OFDM symbol's
//   element t + 64 i per lane, as the fused kernels touch y)}  x  {plain, nontemporal}
//   copy and "read+write" (half the workgroups read buffer A while the other half write B).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <string>

#define CHECK(x)                                                                      \
    do {                                                                              \
        hipError_t e_ = (x);                                                          \
        if (e_ != hipSuccess) {                                                       \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            exit(1);                                                                  \
        }                                                                             \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));
typedef float f2 __attribute__((ext_vector_type(2)));

template <typename T, bool NT>
__device__ __forceinline__ T ld(const T* p) {
    if constexpr (NT) return __builtin_nontemporal_load(p);
    return *p;
}
template <typename T, bool NT>
__device__ __forceinline__ void st(T* p, T v) {
    if constexpr (NT)
        __builtin_nontemporal_store(v, p);
    else
        *p = v;
}

// 16-byte lanes, grid-stride
template <bool NT>
__global__ __launch_bounds__(512) void k_read4(const f4* __restrict__ a, size_t n, float* out) {
    f4 acc = {0, 0, 0, 0};
    for (size_t i = blockIdx.x * 512ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 512) acc += ld<f4, NT>(a + i);
    const float s = acc.x + acc.y + acc.z + acc.w;
    if (s == 12345.f) out[blockIdx.x] = s;  // keep the loads
}
template <bool NT>
__global__ __launch_bounds__(512) void k_write4(f4* __restrict__ a, size_t n, float v) {
    for (size_t i = blockIdx.x * 512ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 512)
        st<f4, NT>(a + i, f4{v, v, v, v});
}

// the fused kernels' pattern: a wave owns one 1024-element complex64 symbol, lane t touches
// elements t + 64 i (16 x 8-byte accesses, each instruction 512 contiguous bytes)
template <bool NT>
__global__ __launch_bounds__(512) void k_read_sym(const f2* __restrict__ a, size_t nsym, float* out) {
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    f2 acc = {0, 0};
    for (size_t s = blockIdx.x * 8ull + w; s < nsym; s += (size_t)gridDim.x * 8) {
        const f2* p = a + s * 1024 + t;
#pragma unroll
        for (int i = 0; i < 16; ++i) acc += ld<f2, NT>(p + 64 * i);
    }
    if (acc.x + acc.y == 12345.f) out[blockIdx.x] = acc.x;
}
template <bool NT>
__global__ __launch_bounds__(512) void k_write_sym(f2* __restrict__ a, size_t nsym, float v) {
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    for (size_t s = blockIdx.x * 8ull + w; s < nsym; s += (size_t)gridDim.x * 8) {
        f2* p = a + s * 1024 + t;
#pragma unroll
        for (int i = 0; i < 16; ++i) st<f2, NT>(p + 64 * i, f2{v, (float)i});
    }
}

// the same symbols with 16-byte lanes: lane t writes elements 2t, 2t+1 + 128 i (8 x 1 KB per wave)
template <bool NT>
__global__ __launch_bounds__(512) void k_write_sym4(f4* __restrict__ a, size_t nsym, float v) {
    const int w = threadIdx.x >> 6, t = threadIdx.x & 63;
    for (size_t s = blockIdx.x * 8ull + w; s < nsym; s += (size_t)gridDim.x * 8) {
        f4* p = a + s * 512 + t;
#pragma unroll
        for (int i = 0; i < 8; ++i) st<f4, NT>(p + 64 * i, f4{v, (float)i, v, v});
    }
}
// one-shot grid (no grid-stride loop): workgroup g writes its own 64 KB chunk, 4 x 16 B per
// thread at a 8 KB stride (the launch-order moving window an elementwise kernel produces)
__global__ __launch_bounds__(512) void k_write_chunk(f4* __restrict__ a, size_t n, float v) {
    const size_t base = (size_t)blockIdx.x * 2048 + threadIdx.x;
#pragma unroll
    for (int i = 0; i < 4; ++i)
        if (base + 512 * i < n) a[base + 512 * i] = f4{v, v, v, (float)i};
}

__global__ __launch_bounds__(512) void k_copy(const f4* __restrict__ a, f4* __restrict__ b, size_t n) {
    for (size_t i = blockIdx.x * 512ull + threadIdx.x; i < n; i += (size_t)gridDim.x * 512) b[i] = a[i];
}

// even workgroups read a, odd workgroups write b
__global__ __launch_bounds__(512) void k_mix(const f4* __restrict__ a, f4* __restrict__ b, size_t n, float* out) {
    const size_t half = gridDim.x / 2;
    const size_t g = blockIdx.x >> 1;
    if (blockIdx.x & 1) {
        for (size_t i = g * 512ull + threadIdx.x; i < n; i += half * 512) __builtin_nontemporal_store(f4{1, 2, 3, 4}, b + i);
    } else {
        f4 acc = {0, 0, 0, 0};
        for (size_t i = g * 512ull + threadIdx.x; i < n; i += half * 512) acc += a[i];
        const float s = acc.x + acc.y + acc.z + acc.w;
        if (s == 12345.f) out[g] = s;
    }
}

template <typename F>
static float timed(F f, int reps) {
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    f();
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    for (int r = 0; r < reps; ++r) f();
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
    return ms / reps;
}

// tools/hbm_probe loop <MiB> <seconds>: write-then-read batches of <MiB> back to back for
// <seconds> (package power / clock sampled outside, tools/ic_power.sh)
static int loop_mode(size_t mb, double seconds) {
    const size_t ns = mb * (1u << 20) / 8192;
    f2* b;
    float* out;
    CHECK(hipMalloc(&b, ns * 8192));
    CHECK(hipMalloc(&out, 1 << 20));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    const int per_batch = (int)(2048 / mb) + 1;
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    double total_ms = 0, bytes = 0;
    while (total_ms < seconds * 1e3) {
        CHECK(hipEventRecord(e0, 0));
        for (int r = 0; r < per_batch; ++r) {
            k_write_sym<false><<<cus * 2, 512>>>(b, ns, 1.f);
            k_read_sym<true><<<cus * 2, 512>>>(b, ns, out);
        }
        CHECK(hipEventRecord(e1, 0));
        CHECK(hipEventSynchronize(e1));
        float ms;
        CHECK(hipEventElapsedTime(&ms, e0, e1));
        total_ms += ms;
        bytes += 2.0 * per_batch * ns * 8192;
    }
    printf("{\"batch_MiB\": %zu, \"seconds\": %.2f, \"write+read_GBps\": %.0f}\n", mb, total_ms / 1e3, bytes / total_ms / 1e6);
    return 0;
}

int main(int argc, char** argv) {
    if (argc >= 4 && std::string(argv[1]) == "loop") return loop_mode(std::stoul(argv[2]), std::stod(argv[3]));
    const size_t nsym = 1000000;
    const size_t bytes = nsym * 1024 * 8;
    const size_t n = bytes / 16;
    f4 *a, *b;
    float* out;
    CHECK(hipMalloc(&a, bytes));
    CHECK(hipMalloc(&b, bytes));
    CHECK(hipMalloc(&out, 1 << 20));
    CHECK(hipMemset(a, 0x3c, bytes));
    int cus = 0;
    CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
    printf("{\"buffer_bytes\": %zu, \"cus\": %d", bytes, cus);
    for (int per_cu : {2, 4, 8}) {
        const int grid = cus * per_cu;
        const double B = (double)bytes / 1e6;  // GB/s from ms
        printf(", \"wg_per_cu_%d\": {", per_cu);
        printf("\"read_x4\": %.0f", B / timed([&] { k_read4<false><<<grid, 512>>>(a, n, out); }, 5));
        printf(", \"read_x4_nt\": %.0f", B / timed([&] { k_read4<true><<<grid, 512>>>(a, n, out); }, 5));
        printf(", \"read_sym\": %.0f", B / timed([&] { k_read_sym<false><<<grid, 512>>>((const f2*)a, nsym, out); }, 5));
        printf(", \"read_sym_nt\": %.0f", B / timed([&] { k_read_sym<true><<<grid, 512>>>((const f2*)a, nsym, out); }, 5));
        printf(", \"write_x4\": %.0f", B / timed([&] { k_write4<false><<<grid, 512>>>(b, n, 1.f); }, 5));
        printf(", \"write_x4_nt\": %.0f", B / timed([&] { k_write4<true><<<grid, 512>>>(b, n, 1.f); }, 5));
        printf(", \"write_sym\": %.0f", B / timed([&] { k_write_sym<false><<<grid, 512>>>((f2*)b, nsym, 1.f); }, 5));
        printf(", \"write_sym_nt\": %.0f", B / timed([&] { k_write_sym<true><<<grid, 512>>>((f2*)b, nsym, 1.f); }, 5));
        printf(", \"write_sym4\": %.0f", B / timed([&] { k_write_sym4<false><<<grid, 512>>>(b, nsym, 1.f); }, 5));
        printf(", \"write_sym4_nt\": %.0f", B / timed([&] { k_write_sym4<true><<<grid, 512>>>(b, nsym, 1.f); }, 5));
        printf(", \"copy\": %.0f", 2 * B / timed([&] { k_copy<<<grid, 512>>>(a, b, n); }, 5));
        printf(", \"read+write_nt\": %.0f}", 2 * B / timed([&] { k_mix<<<2 * grid, 512>>>(a, b, n, out); }, 5));
    }
    // producer -> consumer through the Infinity Cache: write a batch of OFDM symbols, then read
    // it back, batch after batch in one buffer (the fused TX / RX pair at batch granularity)
    printf(", \"write_then_read_batches\": {");
    for (size_t mb : {32, 64, 128, 192, 256, 512, 1024}) {
        const size_t ns = mb * (1u << 20) / 8192;
        const int reps = (int)(8192 / mb) + 1;
        const float tw = timed([&] { k_write_sym<false><<<cus * 2, 512>>>((f2*)b, ns, 1.f); }, reps);
        const float tr = timed([&] { k_read_sym<true><<<cus * 2, 512>>>((const f2*)b, ns, out); }, reps);
        const float tb = timed([&] {
            k_write_sym<false><<<cus * 2, 512>>>((f2*)b, ns, 1.f);
            k_read_sym<true><<<cus * 2, 512>>>((const f2*)b, ns, out);
        }, reps);
        const double by = (double)ns * 8192;
        printf("%s\"%zu MiB\": {\"write_alone\": %.0f, \"read_alone\": %.0f, \"write+read\": %.0f}", mb == 32 ? "" : ", ", mb,
               by / tw / 1e6, by / tr / 1e6, 2 * by / tb / 1e6);
    }
    printf("}");
    printf(", \"write_chunk_oneshot\": %.0f",
           (double)bytes / 1e6 / timed([&] { k_write_chunk<<<(unsigned)((n + 2047) / 2048), 512>>>(b, n, 2.f); }, 5));
    CHECK(hipGetLastError());
    printf("}\n");
    return 0;
}
