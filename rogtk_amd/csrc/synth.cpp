// synth.cpp — seeded synthetic UMI / read generator (host C++, OpenMP).
//
// Frozen spec "synth-v1" (DESIGN.md §Inputs). Every read is a pure function of
// (seed, read index), so any rank can generate any shard [start, start+count)
// of one global dataset with O(count) work and identical bytes regardless of
// world size or thread count:
//   M = max(1, N_total / 10) molecules.
//   read i: rng = xoshiro256** seeded by splitmix64(seed ^ i*PHI);
//           molecule m = lemire(rng(), M)   (family size ~ Binomial(N, 1/M) ≈ Poisson(10))
//           parent UMI bases from splitmix64(seed ^ SALT ^ m*PHI2), 2 bits/base
//           per base: with p_sub substitute one of the 3 other bases uniformly;
//           then with p_n write 'N'; then with p_lower lowercase the byte.
//   template of molecule m (150 bp for H4) from a splitmix64 stream of m;
//   read = template with iid substitutions at p_read_sub.
// Families straddle shards, so multi-GPU runs exercise the cross-shard merge.
#include <cstdint>
#include <cstring>

namespace {

inline uint64_t splitmix64(uint64_t& x) {
    uint64_t z = (x += 0x9E3779B97F4A7C15ull);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    return z ^ (z >> 31);
}

inline uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }

struct Xoshiro256ss {
    uint64_t s[4];
    explicit Xoshiro256ss(uint64_t seed) {
        uint64_t x = seed;
        for (int i = 0; i < 4; ++i) s[i] = splitmix64(x);
    }
    uint64_t next() {
        const uint64_t result = rotl(s[1] * 5, 7) * 9;
        const uint64_t t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3];
        s[2] ^= t;
        s[3] = rotl(s[3], 45);
        return result;
    }
    double uniform() { return (double)(next() >> 11) * 0x1.0p-53; }
};

inline uint64_t lemire(uint64_t r, uint64_t m) {
    return (uint64_t)(((unsigned __int128)r * m) >> 64);
}

constexpr uint64_t PHI = 0x9E3779B97F4A7C15ull;
constexpr uint64_t PHI2 = 0xD1B54A32D192ED03ull;
constexpr uint64_t SALT_UMI = 0x554D495041524E54ull;  // "UMIPARNT"
constexpr uint64_t SALT_TPL = 0x54454D504C415445ull;  // "TEMPLATE"
const char BASES[4] = {'A', 'C', 'G', 'T'};

inline uint64_t molecule_of(uint64_t seed, uint64_t i, uint64_t M, Xoshiro256ss& rng) {
    (void)seed; (void)i;
    return lemire(rng.next(), M);
}

inline uint64_t parent_bits(uint64_t seed, uint64_t m) {
    uint64_t x = seed ^ SALT_UMI ^ (m * PHI2);
    uint64_t a = splitmix64(x);
    return a;
}

// Fill one UMI (bytes) for read i; returns true when the UMI is pure ACGT.
inline bool make_umi(uint64_t n_total, int L, uint64_t seed, double p_sub, double p_n,
                     double p_lower, uint64_t i, uint8_t* out, uint32_t* code) {
    const uint64_t M = n_total / 10 ? n_total / 10 : 1;
    Xoshiro256ss rng(seed ^ (i * PHI));
    const uint64_t m = molecule_of(seed, i, M, rng);
    uint64_t pb = parent_bits(seed, m);
    uint64_t pb2 = 0;
    if (L > 32) { uint64_t x = seed ^ SALT_UMI ^ ((m + 1) * PHI2) ^ 1; pb2 = splitmix64(x); }
    bool regular = true;
    uint32_t c = 0;
    for (int j = 0; j < L; ++j) {
        int b = j < 32 ? (int)((pb >> (2 * j)) & 3) : (int)((pb2 >> (2 * (j - 32))) & 3);
        if (p_sub > 0.0 && rng.uniform() < p_sub) b = (b + 1 + (int)(rng.next() % 3)) & 3;
        uint8_t ch = (uint8_t)BASES[b];
        if (p_n > 0.0 && rng.uniform() < p_n) { ch = 'N'; regular = false; }
        if (p_lower > 0.0 && rng.uniform() < p_lower) { ch = (uint8_t)(ch | 0x20); regular = false; }
        if (out) out[j] = ch;
        c = (c << 2) | (uint32_t)b;
    }
    if (code) *code = c;
    return regular;
}

}  // namespace

extern "C" {

// Fixed-width ASCII UMIs for reads [start, start+count): out[count*L].
void rogtk_synth_umis_ascii(uint64_t n_total, int umi_len, uint64_t seed, double p_sub, double p_n,
                            double p_lower, uint64_t start, uint64_t count, uint8_t* out) {
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < (int64_t)count; ++k)
        make_umi(n_total, umi_len, seed, p_sub, p_n, p_lower, start + (uint64_t)k,
                 out + (uint64_t)k * (uint64_t)umi_len, nullptr);
}

// Packed 2-bit codes (first base most significant) for reads [start, start+count).
// Same reads as rogtk_synth_umis_ascii with p_n = p_lower = 0. umi_len <= 16.
int rogtk_synth_umis_codes(uint64_t n_total, int umi_len, uint64_t seed, double p_sub,
                           uint64_t start, uint64_t count, uint32_t* out) {
    if (umi_len < 1 || umi_len > 16) return 1;
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < (int64_t)count; ++k)
        make_umi(n_total, umi_len, seed, p_sub, 0.0, 0.0, start + (uint64_t)k, nullptr, out + k);
    return 0;
}

// 150-bp style reads (read_len bases, ACGT) for reads [start, start+count):
// molecule template + iid substitutions at p_read_sub. out[count*read_len].
void rogtk_synth_reads(uint64_t n_total, int read_len, uint64_t seed, double p_read_sub,
                       uint64_t start, uint64_t count, uint8_t* out) {
    const uint64_t M = n_total / 10 ? n_total / 10 : 1;
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < (int64_t)count; ++k) {
        const uint64_t i = start + (uint64_t)k;
        Xoshiro256ss rng(seed ^ (i * PHI));
        const uint64_t m = lemire(rng.next(), M);  // same molecule as the read's UMI
        uint64_t x = seed ^ SALT_TPL ^ (m * PHI2);
        uint8_t* o = out + (uint64_t)k * (uint64_t)read_len;
        uint64_t bits = 0;
        Xoshiro256ss mut(seed ^ SALT_TPL ^ (i * PHI2));
        for (int j = 0; j < read_len; ++j) {
            if ((j & 31) == 0) bits = splitmix64(x);
            int b = (int)((bits >> (2 * (j & 31))) & 3);
            if (p_read_sub > 0.0 && mut.uniform() < p_read_sub) b = (b + 1 + (int)(mut.next() % 3)) & 3;
            o[j] = (uint8_t)BASES[b];
        }
    }
}

// Molecule id of each read (ground truth for family statistics in tests).
void rogtk_synth_molecules(uint64_t n_total, uint64_t seed, uint64_t start, uint64_t count, uint64_t* out) {
    const uint64_t M = n_total / 10 ? n_total / 10 : 1;
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < (int64_t)count; ++k) {
        Xoshiro256ss rng(seed ^ ((start + (uint64_t)k) * PHI));
        out[k] = lemire(rng.next(), M);
    }
}

}  // extern "C"
