// sampler.cpp — host generation of the SequenceSamplerData tables.
//
// The reference regenerates the tables on the host at every UpdateKernel from
// one CudaRNG(7539414) stream that continues across passes
// (IndependantSamplingSequenceGenerator, Kernel/Sampler.h:63-85; driver
// SamplingSequenceGeneratorHost::Compute, Sampler.h:36-55): per sequence s,
// 30 1-D draws then 30 (x, y) pairs, stored element-major [k*num_seq + s]
// (Sampler_device.h:20-24).  CudaRNG is cuRAND XORWOW seeded
// curand_init(1234, 7539414, 0) (Base/CudaRandom.cu:27-34); a subsequence is
// 2^67 steps.  We jump straight to pass p's first draw with precomputed
// GF(2) powers of the XORWOW step, so any pass (and any rank) is independent.
#include <cstdint>
#include <cstring>
#include <mutex>
#include <vector>
#include "../../../include/ctl_trace.h"

namespace ctl {
namespace {

struct XorwowState { uint32_t v[5]; uint32_t d; };

struct Gf2Matrix { uint32_t col[160][5]; };

void apply(const Gf2Matrix& M, uint32_t v[5]) {
    uint32_t r[5] = {0, 0, 0, 0, 0};
    for (int w = 0; w < 5; w++) {
        uint32_t bits = v[w];
        while (bits) {
            int b = __builtin_ctz(bits);
            bits &= bits - 1;
            const uint32_t* c = M.col[w * 32 + b];
            r[0] ^= c[0]; r[1] ^= c[1]; r[2] ^= c[2]; r[3] ^= c[3]; r[4] ^= c[4];
        }
    }
    memcpy(v, r, sizeof(r));
}

const std::vector<Gf2Matrix>& step_powers() {   // [k] = (XORWOW step)^(2^k)
    static std::vector<Gf2Matrix> P;
    static std::once_flag once;
    std::call_once(once, [] {
        P.resize(128);
        for (int j = 0; j < 160; j++) {
            uint32_t v[5] = {0, 0, 0, 0, 0};
            v[j >> 5] = 1u << (j & 31);
            uint32_t t = v[0] ^ (v[0] >> 2);
            uint32_t n[5] = {v[1], v[2], v[3], v[4], (v[4] ^ (v[4] << 4)) ^ (t ^ (t << 1))};
            memcpy(P[0].col[j], n, sizeof(n));
        }
        for (int k = 1; k < 128; k++)
            for (int j = 0; j < 160; j++) {
                uint32_t c[5];
                memcpy(c, P[k - 1].col[j], sizeof(c));
                apply(P[k - 1], c);
                memcpy(P[k].col[j], c, sizeof(c));
            }
    });
    return P;
}

XorwowState xorwow_at(uint64_t seed, uint64_t subsequence, uint64_t offset) {
    XorwowState s;
    uint32_t s0 = (uint32_t)seed ^ 0xaad26b49u, s1 = (uint32_t)(seed >> 32) ^ 0xf7dcefddu;
    uint32_t t0 = 1099087573u * s0, t1 = 2591861531u * s1;
    s.d = 6615241u + t1 + t0;
    s.v[0] = 123456789u + t0;
    s.v[1] = 362436069u ^ t0;
    s.v[2] = 521288629u + t1;
    s.v[3] = 88675123u ^ t1;
    s.v[4] = 5783321u + t0;
    const auto& P = step_powers();
    for (int b = 0; b < 61; b++)
        if ((subsequence >> b) & 1) apply(P[67 + b], s.v);
    for (int b = 0; b < 64; b++)
        if ((offset >> b) & 1) apply(P[b], s.v);
    s.d += 362437u * (uint32_t)offset;
    return s;
}

inline float next_uniform(XorwowState& s) {
    uint32_t t = s.v[0] ^ (s.v[0] >> 2);
    s.v[0] = s.v[1]; s.v[1] = s.v[2]; s.v[2] = s.v[3]; s.v[3] = s.v[4];
    s.v[4] = (s.v[4] ^ (s.v[4] << 4)) ^ (t ^ (t << 1));
    s.d += 362437u;
    uint32_t x = s.v[4] + s.d;
    const float kInv = 2.3283064e-10f;                 // CURAND_2POW32_INV
    float f = (float)x * kInv + (kInv / 2.0f);         // curand_uniform
    return f * (1 - 1e-5f);                            // CudaRandom.cu:15
}

}  // namespace

// First XORWOW state of pass `pass` (for the device generator) and the
// GF(2) powers M^(2^k), k < kmax, as kmax x 160 columns x 5 words.
void sampler_pass_state(uint64_t pass, uint32_t nseq, uint32_t len, uint32_t v[5], uint32_t* d) {
    XorwowState s = xorwow_at(1234, 7539414, pass * ((uint64_t)nseq * len * 3));
    memcpy(v, s.v, sizeof(s.v));
    *d = s.d;
}
void sampler_step_powers(uint32_t* out, int kmax) {
    const auto& P = step_powers();
    for (int k = 0; k < kmax; k++) memcpy(out + (size_t)k * 800, P[k].col, 800 * sizeof(uint32_t));
}

// Jumps to a sequence's first draw in two steps: with A = M^(3 len) (one
// sequence's draws), sequence q = 64 qh + ql starts at A^ql A^(64 qh) times the
// pass's first state.  out: [ql = 0..63] A^ql, then [qh = 0..63] A^(64 qh),
// then M^len and M^(len + 2 floor(len / 2)) (where a sequence's 2-D pairs and
// their second half start), 160 columns x 5 words each (130 x 800 words; index
// 0 of each half of the first 128 is the identity).
void sampler_seq_powers(uint32_t* out, uint32_t len) {
    const auto& P = step_powers();
    for (int m = 1; m <= 2; m++) {
        const uint64_t st = m == 1 ? (uint64_t)len : (uint64_t)len + 2ull * (len / 2);
        uint32_t* dst = out + (size_t)(127 + m) * 800;
        for (int j = 0; j < 160; j++) {
            uint32_t v[5] = {0, 0, 0, 0, 0};
            v[j >> 5] = 1u << (j & 31);
            for (int b = 0; b < 64; b++)
                if ((st >> b) & 1) apply(P[b], v);
            memcpy(dst + j * 5, v, sizeof(v));
        }
    }
    const uint64_t steps = 3ull * len;
    Gf2Matrix A, cur, next;
    for (int j = 0; j < 160; j++) {
        uint32_t v[5] = {0, 0, 0, 0, 0};
        v[j >> 5] = 1u << (j & 31);
        for (int b = 0; b < 64; b++)
            if ((steps >> b) & 1) apply(P[b], v);
        memcpy(A.col[j], v, sizeof(v));
    }
    for (int half = 0; half < 2; half++) {
        // step matrix of this half: A, then A^64
        Gf2Matrix S = A;
        if (half == 1)
            for (int j = 0; j < 160; j++)
                for (int r = 1; r < 64; r++) apply(A, S.col[j]);
        memset(&cur, 0, sizeof(cur));
        for (int j = 0; j < 160; j++) cur.col[j][j >> 5] = 1u << (j & 31);   // identity
        for (int i = 0; i < 64; i++) {
            memcpy(out + ((size_t)half * 64 + i) * 800, cur.col, 800 * sizeof(uint32_t));
            for (int j = 0; j < 160; j++) {
                memcpy(next.col[j], cur.col[j], sizeof(next.col[j]));
                apply(S, next.col[j]);
            }
            cur = next;
        }
    }
}

void sampler_tables(uint64_t pass, uint32_t nseq, uint32_t len, float* seq1d, float* seq2d) {
    const uint64_t per_pass = (uint64_t)nseq * len * 3;
    XorwowState s = xorwow_at(1234, 7539414, pass * per_pass);
    for (uint32_t q = 0; q < nseq; q++) {
        for (uint32_t i = 0; i < len; i++) seq1d[(size_t)i * nseq + q] = next_uniform(s);
        for (uint32_t i = 0; i < len; i++) {
            float x = next_uniform(s);
            float y = next_uniform(s);
            seq2d[2 * ((size_t)i * nseq + q)] = x;
            seq2d[2 * ((size_t)i * nseq + q) + 1] = y;
        }
    }
}

}  // namespace ctl

extern "C" CTL_API ctl_status ctl_host_sampler_tables(uint64_t pass_index, uint32_t num_sequences,
                                                      uint32_t sequence_length, float* seq1d, float* seq2d) {
    if (!seq1d || !seq2d || num_sequences == 0 || sequence_length == 0) return CTL_ERR_INVALID;
    ctl::sampler_tables(pass_index, num_sequences, sequence_length, seq1d, seq2d);
    return CTL_OK;
}
