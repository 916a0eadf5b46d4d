// Parity-mode sampling noise generated on the device.
//
// The reference samples with torch.multinomial(p, 1) on CPU (hf_export/
// modeling_t5gemma_voice.py:133-138), which draws V exponential variates per call from
// torch's global CPU generator (SURVEY a14' step 6): the token is the first argmax of
// bf16(p / q). torch 2.10's CPU exponential_ is a serial kernel over the generator's
// MT19937 engine (measured here: every draw of seeds 1..N equals this restatement, see
// tests/test_noise_cpu.py):
//   r64 = (out[2i] << 32) | out[2i+1]        two consecutive 32-bit MT19937 outputs
//   u   = (r64 & (2^53 - 1)) * 2^-53         uniform_real_distribution<double>(0, 1)
//   q   = bf16(float(-log1p(-u)))            transformation::exponential (CPU branch)
// so step s of a row consumes outputs [2 V s, 2 V (s + 1)) of the row's stream.
//
// Drawing them with torch on the host cost 2-4 ms per step and row (14 s of a 19 s C3
// parity generate(), round 4 baseline). Here one workgroup per row runs the MT19937
// recurrence and writes the raw 32-bit outputs to HBM; the sampler turns the pairs of
// the few indices it needs (top-k survivors) into q. The recurrence
//   mt[i] = mt[i + 397] ^ twist(mt[i], mt[i + 1])      (indices mod 624)
// is computed in registers: thread j owns i = j, 227 + j, 454 + j, whose inputs are
// old words or the new word of the SAME thread (i - 227), except mt[0] for i = 623,
// so one twist is one read phase, one write phase and two barriers.
#include "common.h"
#include "t5g_kernels.h"

namespace t5g {

constexpr int MT_N = 624, MT_M = 397, MT_W = MT_N + 1;   // state words + position
constexpr uint32_t MT_UPPER = 0x80000000u, MT_LOWER = 0x7fffffffu, MT_A = 0x9908b0dfu;

__device__ __forceinline__ uint32_t mt_twist(uint32_t cur, uint32_t nxt, uint32_t far) {
    const uint32_t y = (cur & MT_UPPER) | (nxt & MT_LOWER);
    return far ^ (y >> 1) ^ ((y & 1u) ? MT_A : 0u);
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t y) {
    y ^= y >> 11;
    y ^= (y << 7) & 0x9d2c5680u;
    y ^= (y << 15) & 0xefc60000u;
    y ^= y >> 18;
    return y;
}

// One workgroup (256 threads) per row. init[b] = 624 state words + pos (outputs of that
// state already consumed, 1..624; 624 = a twist is due: torch's `left` = 625 - pos).
// Writes outputs [0, n_out) of the row's stream to out[b * out_stride + n] and, for
// s < n_snap, the generator as it stands after n = s * snap_every outputs to
// snap[(b * n_snap + s) * 625] (words + pos, pos in 1..624; the parity host writes the
// snapshot at the row's step count back into torch's generator).
__global__ __launch_bounds__(256) void mt_stream_kernel(const uint32_t* __restrict__ init, long n_out, long out_stride,
                                                        uint32_t* __restrict__ out, long snap_every, int n_snap,
                                                        uint32_t* __restrict__ snap) {
    __shared__ uint32_t mt[MT_N];
    const int b = blockIdx.x, tid = threadIdx.x;
    const uint32_t* src = init + (long)b * MT_W;
    for (int i = tid; i < MT_N; i += 256) mt[i] = src[i];
    const int p0 = (int)min(max(src[MT_N], 0u), (uint32_t)MT_N);
    uint32_t* o = out + (long)b * out_stride;
    uint32_t* sn = snap ? snap + (long)b * n_snap * MT_W : nullptr;
    __syncthreads();
    // state t covers stream indices [start, start + 624) (word i at start + i); a snapshot
    // at stream index n belongs to the state with start < n <= start + 624 (t = 0: n >= 0)
    long start = -(long)p0;
    auto snapshot = [&](bool first) {
        if (!sn) return;
        const long s_hi = min((start + MT_N) / snap_every, (long)n_snap - 1);
        const long s_lo = first ? 0 : start / snap_every + 1;   // start >= 0 past the first state
        for (long s = s_lo; s <= s_hi; ++s) {
            uint32_t* d = sn + s * MT_W;
            for (int i = tid; i < MT_N; i += 256) d[i] = mt[i];
            if (tid == 0) d[MT_N] = (uint32_t)(s * snap_every - start);
        }
    };
    // t = 0: the words still unconsumed in the initial state
    for (int i = p0 + tid; i < MT_N; i += 256)
        if (start + i < n_out) o[start + i] = mt_temper(mt[i]);
    snapshot(true);
    start += MT_N;
    while (start < n_out) {
        // ---- twist (read phase: every input is an old word or this thread's own new word)
        const int j = tid;
        uint32_t n1 = 0, n2 = 0, n3 = 0;
        if (j < MT_N - MT_M) {   // 227
            const uint32_t a0 = mt[j], a1 = mt[j + 1], a2 = mt[j + MT_M];
            const uint32_t b0 = mt[j + 227], b1 = mt[j + 228];
            uint32_t c0 = 0, c1 = 0, z0 = 0, z1 = 0, z2 = 0;
            if (j < MT_N - 454) {   // 170
                c0 = mt[j + 454];
                if (j + 455 < MT_N) c1 = mt[j + 455];
                else { z0 = mt[0]; z1 = mt[1]; z2 = mt[MT_M]; }   // i = 623 needs the new mt[0]
            }
            n1 = mt_twist(a0, a1, a2);
            n2 = mt_twist(b0, b1, n1);
            if (j < MT_N - 454) {
                if (j + 455 >= MT_N) c1 = mt_twist(z0, z1, z2);
                n3 = mt_twist(c0, c1, n2);
            }
        }
        __syncthreads();
        if (j < 227) {
            mt[j] = n1;
            mt[j + 227] = n2;
            if (j < 170) mt[j + 454] = n3;
        }
        __syncthreads();
        // ---- outputs of this state (tempered from the registers), snapshot if one falls here
        if (j < 227) {
            if (start + j < n_out) o[start + j] = mt_temper(n1);
            if (start + 227 + j < n_out) o[start + 227 + j] = mt_temper(n2);
            if (j < 170 && start + 454 + j < n_out) o[start + 454 + j] = mt_temper(n3);
        }
        snapshot(false);
        start += MT_N;
    }
    // a snapshot exactly at n_out with n_out a multiple of 624 past the initial state
    // belongs to the last state above (n <= start + 624 with start the last state's base)
}

int mt_stream(const uint32_t* init, int B, long n_out, long out_stride, uint32_t* out, long snap_every, int n_snap,
              uint32_t* snap, hipStream_t st) {
    if (B <= 0 || n_out < 0) return -1;
    if (!init || !out || out_stride < n_out) return -1;
    if (snap && (snap_every <= 0 || n_snap <= 0)) return -1;
    hipLaunchKernelGGL(mt_stream_kernel, dim3((unsigned)B), dim3(256), 0, st, init, n_out, out_stride, out,
                       snap_every, n_snap, snap);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

__global__ void mt_exp_kernel(const uint32_t* __restrict__ raw, long n, bf16_t* __restrict__ q) {
    const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) q[i] = f2bf(mt_exp_q(raw[2 * i], raw[2 * i + 1]));
}

int mt_exponential(const uint32_t* raw, long n, bf16_t* q, hipStream_t st) {
    if (n <= 0) return 0;
    if (!raw || !q) return -1;
    hipLaunchKernelGGL(mt_exp_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, st, raw, n, q);
    return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace t5g
