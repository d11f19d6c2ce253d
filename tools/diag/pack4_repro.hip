// Stand-alone reduction of the byte-packing miscompile recorded at h264_kernels.hip:140-148
// (VERDICT r2 #8): four 6-tap filter outputs, clamped to 8 bits, OR-ed into one dword as
// `clip255(v) << 8 * j`.  On the MI355X the hpel kernel built this way produced 0xff in bytes
// 2-3 whenever sample 1 clamped from below to 0.  Three packings of the same values are
// compared with a host reference:
//   k_shift_or   -- the original form (clip then shift-or)
//   k_perm       -- the v_perm_b32 form the encoder uses now (pack4)
//   k_masked     -- clip, then `& 0xff` before the shift (what an audit fix would look like)
// plus k_site_recon, the form of the reconstruction stores (h264_kernels.hip k_inter_encode,
// hevc_kernels.hip): clip255(pred + res) << 8 * c, for the audit.
//
//   hipcc --offload-arch=gfx950 -O3 tools/diag/pack4_repro.hip -o /tmp/pack4_repro && /tmp/pack4_repro
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

__device__ __forceinline__ int clip255(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }
__device__ __forceinline__ int tap6(int a, int b, int c, int d, int e, int f) { return a - 5 * b + 20 * c + 20 * d - 5 * e + f; }

// 6-tap half-sample values of 4 neighbouring positions from 9 input samples
__device__ __forceinline__ void taps(const int* s, int* v) {
    for (int j = 0; j < 4; ++j) v[j] = (tap6(s[j], s[j + 1], s[j + 2], s[j + 3], s[j + 4], s[j + 5]) + 16) >> 5;
}

__global__ void k_shift_or(const int* in, uint32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int s[9], v[4];
    for (int k = 0; k < 9; ++k) s[k] = in[i * 9 + k];
    taps(s, v);
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) w |= (uint32_t)clip255(v[j]) << (8 * j);
    out[i] = w;
}

__global__ void k_perm(const int* in, uint32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int s[9], v[4];
    for (int k = 0; k < 9; ++k) s[k] = in[i * 9 + k];
    taps(s, v);
    const uint32_t lo = __builtin_amdgcn_perm((uint32_t)clip255(v[1]), (uint32_t)clip255(v[0]), 0x0c0c0400u);
    const uint32_t hi = __builtin_amdgcn_perm((uint32_t)clip255(v[3]), (uint32_t)clip255(v[2]), 0x0c0c0400u);
    out[i] = __builtin_amdgcn_perm(hi, lo, 0x05040100u);
}

__global__ void k_masked(const int* in, uint32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    int s[9], v[4];
    for (int k = 0; k < 9; ++k) s[k] = in[i * 9 + k];
    taps(s, v);
    uint32_t w = 0;
#pragma unroll
    for (int j = 0; j < 4; ++j) w |= ((uint32_t)clip255(v[j]) & 0xffu) << (8 * j);
    out[i] = w;
}

__global__ void k_site_recon(const int* in, uint32_t* out, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint32_t w = 0;
#pragma unroll
    for (int c = 0; c < 4; ++c) w |= (uint32_t)clip255(in[i * 9 + c] + in[i * 9 + 4 + c]) << (8 * c);
    out[i] = w;
}

static int clip_h(int v) { return v < 0 ? 0 : (v > 255 ? 255 : v); }

int main() {
    const int n = 1 << 20;
    std::vector<int> in((size_t)n * 9);
    srand(7);
    for (auto& x : in) x = (rand() % 3 == 0) ? (rand() % 2 ? 0 : 255) : rand() % 256;  // edges make clamps likely
    for (int i = 0; i < n; i += 7) in[(size_t)i * 9 + 4] = 255, in[(size_t)i * 9 + 3] = 0;
    std::vector<uint32_t> ref(n), ref_site(n);
    for (int i = 0; i < n; ++i) {
        const int* s = &in[(size_t)i * 9];
        uint32_t w = 0, ws = 0;
        for (int j = 0; j < 4; ++j) {
            const int t = s[j] - 5 * s[j + 1] + 20 * s[j + 2] + 20 * s[j + 3] - 5 * s[j + 4] + s[j + 5];
            w |= (uint32_t)clip_h((t + 16) >> 5) << (8 * j);
            ws |= (uint32_t)clip_h(s[j] + s[4 + j]) << (8 * j);  // site form: pred + residual
        }
        ref[i] = w;
        ref_site[i] = ws;
    }
    int* d_in;
    uint32_t* d_out;
    if (hipMalloc(&d_in, in.size() * sizeof(int)) != hipSuccess || hipMalloc(&d_out, n * sizeof(uint32_t)) != hipSuccess)
        return 2;
    (void)hipMemcpy(d_in, in.data(), in.size() * sizeof(int), hipMemcpyHostToDevice);
    struct K {
        const char* name;
        void (*fn)(const int*, uint32_t*, int);
        const std::vector<uint32_t>* want;
    } ks[] = {{"k_shift_or", k_shift_or, &ref}, {"k_perm", k_perm, &ref}, {"k_masked", k_masked, &ref},
              {"k_site_recon", k_site_recon, &ref_site}};
    int rc = 0;
    std::vector<uint32_t> got(n);
    for (auto& k : ks) {
        hipLaunchKernelGGL(k.fn, dim3((n + 255) / 256), dim3(256), 0, 0, d_in, d_out, n);
        if (hipDeviceSynchronize() != hipSuccess) return 3;
        (void)hipMemcpy(got.data(), d_out, n * sizeof(uint32_t), hipMemcpyDeviceToHost);
        int bad = 0, first = -1;
        for (int i = 0; i < n; ++i)
            if (got[i] != (*k.want)[i]) {
                if (first < 0) first = i;
                ++bad;
            }
        std::printf("%-14s mismatches %d / %d", k.name, bad, n);
        if (first >= 0) std::printf("  first at %d: got %08x want %08x", first, got[first], (*k.want)[first]);
        std::printf("\n");
        rc |= bad != 0 && k.fn != k_shift_or;
    }
    (void)hipFree(d_in);
    (void)hipFree(d_out);
    return rc;
}
