// encode.cpp — host encoders (include/vortex_enc.h): restatements of the reference ENCODERS,
// used to synthesise inputs in the exact layouts the reference writes.  Not on the decode path.
// Built with -ffp-contract=off and without fast-math: the ALP encoder must make the same
// round-trip decisions as alp/mod.rs (encode_single_unchecked / decode_single).
#include "../../include/vortex_enc.h"

#include <algorithm>
#include <cmath>
#include <cstring>
#include <limits>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

int ptype_width(int p) {
    switch (p) {
    case 0: case 4: return 1;
    case 1: case 5: case 8: return 2;
    case 2: case 6: case 9: return 4;
    default: return 8;
    }
}

constexpr int FL_ORDER[8] = {0, 4, 2, 6, 1, 5, 3, 7};
inline int fl_index(int row, int lane) { return FL_ORDER[row / 8] * 16 + (row % 8) * 128 + lane; }

// fastlanes 0.1.8 BitPacking::unchecked_pack
template <typename E>
void pack_block(unsigned W, const E* in, E* packed) {
    constexpr unsigned T = 8 * sizeof(E), LANES = 1024 / T;
    if (W == 0) return;
    if (W == T) {
        for (unsigned l = 0; l < LANES; l++)
            for (unsigned r = 0; r < T; r++) packed[LANES * r + l] = in[fl_index(r, l)];
        return;
    }
    const E mask = E((E(1) << W) - 1);
    for (unsigned l = 0; l < LANES; l++) {
        E tmp = 0;
        for (unsigned r = 0; r < T; r++) {
            const E src = E(in[fl_index(r, l)] & mask);
            const unsigned shift = (r * W) % T;
            tmp = r == 0 ? src : E(tmp | E(src << shift));
            const unsigned cur = (r * W) / T, nxt = ((r + 1) * W) / T;
            if (nxt > cur) {
                packed[LANES * cur + l] = tmp;
                const unsigned rem = ((r + 1) * W) % T;
                tmp = rem ? E(src >> (W - rem)) : E(0);
            }
        }
    }
}

template <typename E>
uint64_t bitpack_t(unsigned W, const E* v, uint64_t n, uint8_t* packed) {
    if (W == 0) return 0;
    const uint64_t nblk = (n + 1023) / 1024, full = n / 1024, bb = 128ull * W;
    for (uint64_t b = 0; b < full; b++) pack_block<E>(W, v + b * 1024, reinterpret_cast<E*>(packed + b * bb));
    if (nblk != full) {
        E last[1024] = {};
        std::memcpy(last, v + full * 1024, (n % 1024) * sizeof(E));
        pack_block<E>(W, last, reinterpret_cast<E*>(packed + full * bb));
    }
    return nblk * bb;
}

template <typename E>
void bit_width_freq(const E* v, uint64_t n, std::vector<uint64_t>& freq) {
    constexpr int T = 8 * sizeof(E);
    freq.assign(T + 1, 0);
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t x = uint64_t(v[i]);
        freq[x ? 64 - __builtin_clzll(x) : 0]++;
    }
}

template <typename E> E load(const void* p, uint64_t i) { return static_cast<const E*>(p)[i]; }

uint64_t as_u64(const void* p, int w, uint64_t i) {
    switch (w) {
    case 1: return load<uint8_t>(p, i);
    case 2: return load<uint16_t>(p, i);
    case 4: return load<uint32_t>(p, i);
    default: return load<uint64_t>(p, i);
    }
}

// ---- ALP (alp/mod.rs) ------------------------------------------------------------------
const double F10D[24] = {
    1.0, 10.0, 100.0, 1000.0, 10000.0, 100000.0, 1000000.0, 10000000.0, 100000000.0,
    1000000000.0, 10000000000.0, 100000000000.0, 1000000000000.0, 10000000000000.0,
    100000000000000.0, 1000000000000000.0, 10000000000000000.0, 100000000000000000.0,
    1000000000000000000.0, 10000000000000000000.0, 100000000000000000000.0,
    1000000000000000000000.0, 10000000000000000000000.0, 100000000000000000000000.0};
const double IF10D[24] = {
    1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001, 0.00000001, 0.000000001,
    0.0000000001, 0.00000000001, 0.000000000001, 0.0000000000001, 0.00000000000001,
    0.000000000000001, 0.0000000000000001, 0.00000000000000001, 0.000000000000000001,
    0.0000000000000000001, 0.00000000000000000001, 0.000000000000000000001,
    0.0000000000000000000001, 0.00000000000000000000001};
const float F10F[11] = {1.0f, 10.0f, 100.0f, 1000.0f, 10000.0f, 100000.0f, 1000000.0f,
                        10000000.0f, 100000000.0f, 1000000000.0f, 10000000000.0f};
const float IF10F[11] = {1.0f, 0.1f, 0.01f, 0.001f, 0.0001f, 0.00001f, 0.000001f,
                         0.0000001f, 0.00000001f, 0.000000001f, 0.0000000001f};

template <typename F> struct Alp;
template <> struct Alp<double> {
    using I = int64_t;
    static constexpr int MAX_EXPONENT = 18;
    static constexpr double SWEET = double(1ull << 52) + double(1ull << 51);
    static double f10(int i) { return F10D[i]; }
    static double if10(int i) { return IF10D[i]; }
};
template <> struct Alp<float> {
    using I = int32_t;
    static constexpr int MAX_EXPONENT = 10;
    static constexpr float SWEET = float(1u << 23) + float(1u << 22);
    static float f10(int i) { return F10F[i]; }
    static float if10(int i) { return IF10F[i]; }
};

// Rust `as` float -> int: saturating, NaN -> 0.
template <typename I, typename F> I sat_cast(F x) {
    if (std::isnan(x)) return 0;
    if (x >= F(std::numeric_limits<I>::max())) return std::numeric_limits<I>::max();
    if (x <= F(std::numeric_limits<I>::min())) return std::numeric_limits<I>::min();
    return I(x);
}

template <typename F> typename Alp<F>::I encode_single_unchecked(F v, int e, int f) {
    F x = v * Alp<F>::f10(e);
    x = x * Alp<F>::if10(f);
    x = (x + Alp<F>::SWEET) - Alp<F>::SWEET;  // fast_round
    return sat_cast<typename Alp<F>::I>(x);
}
template <typename F> F decode_single(typename Alp<F>::I enc, int e, int f) {
    F x = F(enc) * Alp<F>::f10(f);
    return x * Alp<F>::if10(e);
}

// encode_chunk_unchecked (alp/mod.rs:173-246), including the fill-value logic.
template <typename F>
void encode_chunk(const F* chunk, uint64_t clen, int e, int f, std::vector<typename Alp<F>::I>& enc,
                  std::vector<uint64_t>& pidx, std::vector<F>& pval, bool& has_fill,
                  typename Alp<F>::I& fill) {
    using I = typename Alp<F>::I;
    const uint64_t num_prev_encoded = enc.size();
    const uint64_t num_prev_patches = pidx.size();
    const bool had_fill = has_fill;
    uint64_t chunk_patch_count = 0;
    for (uint64_t i = 0; i < clen; i++) {
        const I x = encode_single_unchecked<F>(chunk[i], e, f);
        const F d = decode_single<F>(x, e, f);
        chunk_patch_count += (d != chunk[i]);
        enc.push_back(x);
    }
    if (chunk_patch_count > 0) {
        for (uint64_t i = num_prev_encoded; i < enc.size(); i++) {
            const F d = decode_single<F>(enc[i], e, f);
            if (d != chunk[i - num_prev_encoded]) {
                pidx.push_back(i);
                pval.push_back(chunk[i - num_prev_encoded]);
            }
        }
    }
    if (!has_fill && (num_prev_encoded + chunk_patch_count < enc.size())) {
        for (uint64_t i = num_prev_encoded; i < enc.size(); i++) {
            if (i >= pidx.size() || pidx[i] != i) {
                fill = enc[i];
                has_fill = true;
                break;
            }
        }
    }
    if (has_fill) {
        const uint64_t start = had_fill ? num_prev_patches : 0;
        for (uint64_t k = start; k < pidx.size(); k++) enc[pidx[k]] = fill;
    }
}

template <typename F>
void alp_encode_all(const F* values, uint64_t n, int e, int f, std::vector<typename Alp<F>::I>& enc,
                    std::vector<uint64_t>& pidx, std::vector<F>& pval) {
    using I = typename Alp<F>::I;
    enc.clear(); pidx.clear(); pval.clear();
    enc.reserve(n);
    bool has_fill = false;
    I fill = 0;
    const uint64_t chunk = (32 << 10) / sizeof(I);
    for (uint64_t s = 0; s < n; s += chunk)
        encode_chunk<F>(values + s, std::min<uint64_t>(chunk, n - s), e, f, enc, pidx, pval, has_fill, fill);
}

template <typename F>
uint64_t estimate_size(const std::vector<typename Alp<F>::I>& enc, uint64_t n_patches) {
    using I = typename Alp<F>::I;
    uint64_t bits;
    if (enc.empty()) {
        bits = 8 * sizeof(I);
    } else {
        const auto mm = std::minmax_element(enc.begin(), enc.end());
        const I mn = *mm.first, mx = *mm.second;
        I range;
        if (__builtin_sub_overflow(mx, mn, &range)) {
            bits = 8 * sizeof(I);
        } else {
            const uint64_t r = uint64_t(range);
            bits = r == 0 ? 0 : uint64_t(64 - __builtin_clzll(r));
        }
    }
    return (enc.size() * bits + 7) / 8 + n_patches * (sizeof(F) + sizeof(uint16_t));
}

template <typename F>
void find_best_exponents(const F* values, uint64_t n, int& be, int& bf) {
    std::vector<F> sample;
    const F* s = values;
    uint64_t sn = n;
    if (n > 32) {
        const uint64_t step = n / 32;
        for (uint64_t i = 0; i < n; i += step) sample.push_back(values[i]);
        s = sample.data();
        sn = sample.size();
    }
    be = 0; bf = 0;
    uint64_t best = std::numeric_limits<uint64_t>::max();
    std::vector<typename Alp<F>::I> enc;
    std::vector<uint64_t> pidx;
    std::vector<F> pval;
    for (int e = Alp<F>::MAX_EXPONENT - 1; e >= 0; e--) {
        for (int f = 0; f < e; f++) {
            alp_encode_all<F>(s, sn, e, f, enc, pidx, pval);
            const uint64_t size = estimate_size<F>(enc, pidx.size());
            if (size < best) {
                best = size; be = e; bf = f;
            } else if (size == best && e - f < be - bf) {
                be = e; bf = f;
            }
        }
    }
}

template <typename F>
uint64_t alp_encode_t(const F* values, uint64_t n, uint8_t* e, uint8_t* f, typename Alp<F>::I* encoded,
                      uint64_t* patch_idx, F* patch_vals, uint64_t cap) {
    int be, bf;
    find_best_exponents<F>(values, n, be, bf);
    std::vector<typename Alp<F>::I> enc;
    std::vector<uint64_t> pidx;
    std::vector<F> pval;
    alp_encode_all<F>(values, n, be, bf, enc, pidx, pval);
    *e = uint8_t(be);
    *f = uint8_t(bf);
    // (an empty vector's data() may be null: memcpy from it is undefined even for 0 bytes)
    if (n) std::memcpy(encoded, enc.data(), n * sizeof(typename Alp<F>::I));
    const uint64_t m = std::min<uint64_t>(cap, pidx.size());
    if (m) {
        std::memcpy(patch_idx, pidx.data(), m * 8);
        std::memcpy(patch_vals, pval.data(), m * sizeof(F));
    }
    return pidx.size();
}

// ---- ALP-RD (alp_rd/mod.rs:140-352) -----------------------------------------------------
template <typename F, typename U>
uint64_t alprd_encode_t(const F* values, uint64_t n, uint8_t* rbw_out, uint16_t* dict, uint8_t* dict_len,
                        uint16_t* left, U* right, uint64_t* exc_pos, uint16_t* exc, uint64_t cap) {
    constexpr int BITS = 8 * sizeof(F);
    std::vector<U> sample;
    const uint64_t step = n > 8192 ? n / 8192 : 1;
    for (uint64_t i = 0; i < n; i += step) {
        U b;
        std::memcpy(&b, &values[i], sizeof(F));
        sample.push_back(b);
    }
    auto bit_width = [](uint64_t v) -> int { return v == 0 ? 1 : 64 - __builtin_clzll(v); };
    double best_size = std::numeric_limits<double>::max();
    int best_rbw = BITS - 1;
    std::vector<uint16_t> best_codes;
    for (int p = 1; p <= 16; p++) {
        const int rbw = BITS - p;
        std::unordered_map<uint16_t, uint64_t> counts;
        for (U b : sample) counts[uint16_t(b >> rbw)]++;
        std::vector<std::pair<uint16_t, uint64_t>> sorted(counts.begin(), counts.end());
        std::sort(sorted.begin(), sorted.end(), [](auto& a, auto& b) {
            return a.second != b.second ? a.second > b.second : a.first < b.first;
        });
        std::vector<uint16_t> codes;
        uint64_t exc_count = 0;
        for (size_t i = 0; i < sorted.size(); i++) {
            if (i < 8) codes.push_back(sorted[i].first); else exc_count += sorted[i].second;
        }
        const int lbw = bit_width(codes.size() - 1);
        const double size = double(rbw) + double(lbw) + double(exc_count * 32) / double(sample.size());
        if (size < best_size) {
            best_size = size;
            best_rbw = rbw;
            best_codes = codes;
        }
    }
    *rbw_out = uint8_t(best_rbw);
    *dict_len = uint8_t(best_codes.size());
    for (size_t i = 0; i < best_codes.size(); i++) dict[i] = best_codes[i];
    const U rmask = U((U(1) << best_rbw) - 1);
    uint64_t ne = 0;
    for (uint64_t i = 0; i < n; i++) {
        U b;
        std::memcpy(&b, &values[i], sizeof(F));
        right[i] = U(b & rmask);
        const uint16_t l = uint16_t(b >> best_rbw);
        int code = -1;
        for (size_t k = 0; k < best_codes.size(); k++)
            if (best_codes[k] == l) { code = int(k); break; }
        if (code < 0) {
            if (ne < cap) { exc_pos[ne] = i; exc[ne] = l; }
            ne++;
            left[i] = 0;
        } else {
            left[i] = uint16_t(code);
        }
    }
    return ne;
}

}  // namespace

extern "C" {

uint64_t vxe_bitpack(int ptype, unsigned W, const void* v, uint64_t n, void* packed) {
    uint8_t* p = static_cast<uint8_t*>(packed);
    switch (ptype_width(ptype)) {
    case 1: return bitpack_t<uint8_t>(W, static_cast<const uint8_t*>(v), n, p);
    case 2: return bitpack_t<uint16_t>(W, static_cast<const uint16_t*>(v), n, p);
    case 4: return bitpack_t<uint32_t>(W, static_cast<const uint32_t*>(v), n, p);
    default: return bitpack_t<uint64_t>(W, static_cast<const uint64_t*>(v), n, p);
    }
}

static void freq_of(int ptype, const void* v, uint64_t n, std::vector<uint64_t>& freq) {
    switch (ptype_width(ptype)) {
    case 1: bit_width_freq(static_cast<const uint8_t*>(v), n, freq); break;
    case 2: bit_width_freq(static_cast<const uint16_t*>(v), n, freq); break;
    case 4: bit_width_freq(static_cast<const uint32_t*>(v), n, freq); break;
    default: bit_width_freq(static_cast<const uint64_t*>(v), n, freq); break;
    }
}

unsigned vxe_best_bit_width(int ptype, const void* v, uint64_t n) {
    std::vector<uint64_t> freq;
    freq_of(ptype, v, n, freq);
    const uint64_t bpe = uint64_t(ptype_width(ptype)) + 4;
    uint64_t len = 0;
    for (auto x : freq) len += x;
    uint64_t num_packed = 0, best_cost = len * bpe;
    unsigned best = 0;
    for (unsigned bw = 0; bw < freq.size(); bw++) {
        const uint64_t packed_cost = (bw * len + 7) / 8;
        num_packed += freq[bw];
        const uint64_t cost = (len - num_packed) * bpe + packed_cost;
        if (cost < best_cost) { best_cost = cost; best = bw; }
    }
    return best;
}

unsigned vxe_min_patchless_bit_width(int ptype, const void* v, uint64_t n) {
    std::vector<uint64_t> freq;
    freq_of(ptype, v, n, freq);
    unsigned m = 0;
    for (unsigned bw = 0; bw < freq.size(); bw++)
        if (freq[bw]) m = bw;
    return m;
}

uint64_t vxe_gather_patches(int ptype, unsigned W, const void* v, uint64_t n, uint64_t* idx, void* pv,
                            uint64_t cap) {
    const int w = ptype_width(ptype);
    uint64_t c = 0;
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t x = as_u64(v, w, i);
        const unsigned bits = x ? unsigned(64 - __builtin_clzll(x)) : 0;
        if (bits > W) {
            if (c < cap) {
                idx[c] = i;
                std::memcpy(static_cast<uint8_t*>(pv) + c * w, static_cast<const uint8_t*>(v) + i * w, w);
            }
            c++;
        }
    }
    return c;
}

int vxe_for_compress(int ptype, const void* v, uint64_t n, void* encoded, uint64_t* reference, unsigned* shift) {
    const int w = ptype_width(ptype);
    const bool sgn = ptype >= 4 && ptype <= 7;
    const unsigned T = 8u * w;
    const uint64_t mask = w == 8 ? ~0ull : ((1ull << T) - 1);
    // min (signed or unsigned) and min trailing zeros (stats/mod.rs:178-189; tz(0) = T)
    int64_t smin = 0;
    uint64_t umin = 0;
    unsigned tz = T;
    for (uint64_t i = 0; i < n; i++) {
        uint64_t x = as_u64(v, w, i);
        int64_t sx = sgn ? int64_t(x << (64 - T)) >> (64 - T) : int64_t(x);
        if (i == 0 || (sgn ? sx < smin : x < umin)) { smin = sx; umin = x; }
        const unsigned t = x ? unsigned(__builtin_ctzll(x)) : T;
        if (t < tz) tz = t;
    }
    const uint64_t ref = (sgn ? uint64_t(smin) : umin) & mask;
    *reference = ref;
    *shift = tz;
    if (tz >= T) return 1;  // all zeros: ConstantArray in the reference
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t x = as_u64(v, w, i);
        uint64_t d = (x - ref) & mask;
        if (sgn && tz > 0) {
            // signed: (v.wrapping_sub(min)) >> shift is an arithmetic shift in the signed type
            int64_t sd = int64_t(d << (64 - T)) >> (64 - T);
            d = uint64_t(sd >> tz) & mask;
        } else {
            d >>= tz;
        }
        std::memcpy(static_cast<uint8_t*>(encoded) + i * w, &d, w);
    }
    return 0;
}

void vxe_delta_compress(int ptype, const void* values, uint64_t n, void* bases, void* deltas) {
    const int w = ptype_width(ptype);
    const unsigned T = 8u * w, LANES = 1024 / T;
    const uint64_t mask = w == 8 ? ~0ull : ((1ull << T) - 1);
    const uint64_t nchunks = n / 1024;
    uint64_t nb = 0;
    auto put = [&](void* p, uint64_t i, uint64_t x) { std::memcpy(static_cast<uint8_t*>(p) + i * w, &x, w); };
    std::vector<uint64_t> tr(1024);
    for (uint64_t c = 0; c < nchunks; c++) {
        // transposed[i] = input[transpose(i)]
        for (unsigned i = 0; i < 1024; i++) {
            const unsigned lane = i % 16, order = (i / 16) % 8, row = i / 128;
            tr[i] = as_u64(values, w, c * 1024 + lane * 64 + FL_ORDER[order] * 8 + row);
        }
        for (unsigned l = 0; l < LANES; l++) put(bases, nb + l, tr[l]);
        for (unsigned l = 0; l < LANES; l++) {
            uint64_t prev = tr[l];
            for (unsigned r = 0; r < T; r++) {
                const unsigned idx = fl_index(int(r), int(l));
                const uint64_t nx = tr[idx];
                put(deltas, c * 1024 + idx, (nx - prev) & mask);
                prev = nx;
            }
        }
        nb += LANES;
    }
    const uint64_t rem = n % 1024;
    if (rem) {
        uint64_t base = as_u64(values, w, n - rem);
        put(bases, nb, base);
        for (uint64_t i = n - rem; i < n; i++) {
            const uint64_t x = as_u64(values, w, i);
            put(deltas, i, (x - base) & mask);
            base = x;
        }
    }
}

void vxe_zigzag_encode(int in_ptype, const void* values, uint64_t n, void* out) {
    const int w = ptype_width(in_ptype);
    const unsigned T = 8u * w;
    const uint64_t mask = w == 8 ? ~0ull : ((1ull << T) - 1);
    for (uint64_t i = 0; i < n; i++) {
        const uint64_t x = as_u64(values, w, i);
        const int64_t sx = int64_t(x << (64 - T)) >> (64 - T);
        const uint64_t z = ((uint64_t(sx) << 1) ^ uint64_t(sx >> 63)) & mask;
        std::memcpy(static_cast<uint8_t*>(out) + i * w, &z, w);
    }
}

uint64_t vxe_alp_encode_f64(const double* values, uint64_t n, uint8_t* e, uint8_t* f, int64_t* encoded,
                            uint64_t* patch_idx, double* patch_vals, uint64_t cap) {
    return alp_encode_t<double>(values, n, e, f, encoded, patch_idx, patch_vals, cap);
}
uint64_t vxe_alp_encode_f32(const float* values, uint64_t n, uint8_t* e, uint8_t* f, int32_t* encoded,
                            uint64_t* patch_idx, float* patch_vals, uint64_t cap) {
    return alp_encode_t<float>(values, n, e, f, encoded, patch_idx, patch_vals, cap);
}

uint64_t vxe_alprd_encode_f64(const double* values, uint64_t n, uint8_t* rbw, uint16_t* dict, uint8_t* dict_len,
                              uint16_t* left, uint64_t* right, uint64_t* exc_pos, uint16_t* exc, uint64_t cap) {
    return alprd_encode_t<double, uint64_t>(values, n, rbw, dict, dict_len, left, right, exc_pos, exc, cap);
}
uint64_t vxe_alprd_encode_f32(const float* values, uint64_t n, uint8_t* rbw, uint16_t* dict, uint8_t* dict_len,
                              uint16_t* left, uint32_t* right, uint64_t* exc_pos, uint16_t* exc, uint64_t cap) {
    return alprd_encode_t<float, uint32_t>(values, n, rbw, dict, dict_len, left, right, exc_pos, exc, cap);
}

uint64_t vxe_dict_encode(int vw, const void* values, uint64_t n, uint64_t* codes, void* dict_values, uint64_t cap) {
    std::unordered_map<std::string, uint64_t> lut;
    uint64_t nd = 0;
    const uint8_t* v = static_cast<const uint8_t*>(values);
    for (uint64_t i = 0; i < n; i++) {
        std::string key(reinterpret_cast<const char*>(v + i * vw), vw);
        auto it = lut.find(key);
        if (it == lut.end()) {
            it = lut.emplace(key, nd).first;
            if (nd < cap) std::memcpy(static_cast<uint8_t*>(dict_values) + nd * vw, v + i * vw, vw);
            nd++;
        }
        codes[i] = it->second;
    }
    return nd;
}

uint64_t vxe_runend_encode(int vw, const void* values, uint64_t n, uint64_t* ends, void* run_values) {
    const uint8_t* v = static_cast<const uint8_t*>(values);
    uint64_t r = 0;
    for (uint64_t i = 0; i < n; i++) {
        if (i == 0 || std::memcmp(v + i * vw, v + (i - 1) * vw, vw) != 0) {
            if (i) ends[r - 1] = i;
            std::memcpy(static_cast<uint8_t*>(run_values) + r * vw, v + i * vw, vw);
            r++;
        }
    }
    if (r) ends[r - 1] = n;
    return r;
}

void vxe_fsst_train(const uint8_t* heap, const int64_t* offsets, uint64_t n, vxe_fsst_table* t) {
    // Count substrings of length 1..8 over a bounded sample of strings; pick the 255 with the
    // largest gain = count * len, single bytes promoted x8 (the FSST trainer's heuristic that
    // fsst-rs follows: "promoting single-byte symbols (*8) helps reduce exception rates and
    // increases [de]compression speed"); greedily discounting overlaps is skipped.
    std::unordered_map<uint64_t, uint64_t> cnt;  // key = len<<56 | bytes (len <= 7) ; len 8 hashed
    std::unordered_map<uint64_t, uint64_t> cnt8;
    uint64_t sampled = 0;
    const uint64_t step = n > 20000 ? n / 20000 : 1;
    for (uint64_t s = 0; s < n && sampled < (1u << 20); s += step) {
        const uint8_t* p = heap + offsets[s];
        const int64_t L = offsets[s + 1] - offsets[s];
        sampled += uint64_t(L);
        for (int64_t i = 0; i < L; i++) {
            uint64_t key = 0;
            for (int len = 1; len <= 8 && i + len <= L; len++) {
                key |= uint64_t(p[i + len - 1]) << (8 * (len - 1));
                if (len < 8) cnt[(uint64_t(len) << 56) | key]++;
                else cnt8[key]++;
            }
        }
    }
    struct Cand { uint64_t bytes; uint8_t len; uint64_t gain; };
    std::vector<Cand> c;
    for (auto& kv : cnt) {
        const uint8_t len = uint8_t(kv.first >> 56);
        c.push_back({kv.first & ((1ull << 56) - 1), len, kv.second * len * (len == 1 ? 8u : 1u)});
    }
    for (auto& kv : cnt8) c.push_back({kv.first, 8, kv.second * 8});
    std::sort(c.begin(), c.end(), [](const Cand& a, const Cand& b) {
        return a.gain != b.gain ? a.gain > b.gain : (a.len != b.len ? a.len > b.len : a.bytes < b.bytes);
    });
    t->n_symbols = 0;
    for (size_t i = 0; i < c.size() && t->n_symbols < 255; i++) {
        t->symbols[t->n_symbols] = c[i].bytes;
        t->lens[t->n_symbols] = c[i].len;
        t->n_symbols++;
    }
}

uint64_t vxe_fsst_compress(const vxe_fsst_table* t, const uint8_t* heap, const int64_t* offsets, uint64_t n,
                           uint8_t* codes, uint64_t cap, int32_t* code_offsets) {
    // bucket multi-byte symbols by their first two bytes, longest first; single bytes direct
    std::vector<std::vector<int>> b2(65536);
    int single[256];
    std::fill(single, single + 256, -1);
    for (uint32_t s = 0; s < t->n_symbols; s++) {
        if (t->lens[s] == 1) {
            if (single[t->symbols[s] & 0xFF] < 0) single[t->symbols[s] & 0xFF] = int(s);
        } else {
            b2[t->symbols[s] & 0xFFFF].push_back(int(s));
        }
    }
    for (auto& v : b2)
        std::stable_sort(v.begin(), v.end(), [&](int a, int b) { return t->lens[a] > t->lens[b]; });
    uint64_t o = 0;
    code_offsets[0] = 0;
    for (uint64_t s = 0; s < n; s++) {
        const uint8_t* p = heap + offsets[s];
        const int64_t L = offsets[s + 1] - offsets[s];
        int64_t i = 0;
        while (i < L) {
            int code = -1, clen = 1;
            if (i + 1 < L) {
                for (int sid : b2[p[i] | (p[i + 1] << 8)]) {
                    const int sl = t->lens[sid];
                    if (i + sl <= L && std::memcmp(p + i, &t->symbols[sid], sl) == 0) {
                        code = sid; clen = sl; break;
                    }
                }
            }
            if (code < 0) code = single[p[i]];
            if (o + 2 > cap) return UINT64_MAX;
            if (code < 0) {
                codes[o++] = 255;
                codes[o++] = p[i];
                i += 1;
            } else {
                codes[o++] = uint8_t(code);
                i += clen;
            }
        }
        code_offsets[s + 1] = int32_t(o);
    }
    return o;
}

uint64_t vxe_roaring_bool_encode(const uint8_t* bits, uint64_t len, uint8_t* out, uint64_t cap) {
    // Containers of 2^16 positions keyed by the high 16 bits; a container starts as an array
    // (<= 4096 values) or a bitset, and run_optimize turns it into runs when the run form
    // serializes smaller (array: 2 + 4 r < 2 + 2 card; bitset: 2 + 4 r < 8192).
    enum Kind { ARRAY, BITSET, RUN };
    struct Cont {
        uint16_t key;
        Kind kind;
        uint32_t card;
        std::vector<uint16_t> vals;                      // array values
        std::vector<std::pair<uint16_t, uint16_t>> runs; // (start, length - 1)
        uint64_t words[1024];
        uint64_t bytes() const { return kind == ARRAY ? 2ull * card : kind == BITSET ? 8192 : 2 + 4ull * runs.size(); }
    };
    std::vector<Cont> cs;
    uint64_t card_total = 0;
    for (uint64_t base = 0; base < len; base += 65536) {
        const uint64_t end = std::min<uint64_t>(len, base + 65536);
        Cont c{};
        c.key = uint16_t(base >> 16);
        for (uint64_t i = base; i < end; i++) {
            if (!((bits[i >> 3] >> (i & 7)) & 1)) continue;
            const uint16_t x = uint16_t(i - base);
            c.words[x >> 6] |= 1ull << (x & 63);
            c.vals.push_back(x);
            if (!c.runs.empty() && uint32_t(c.runs.back().first) + c.runs.back().second + 1 == x)
                c.runs.back().second++;
            else
                c.runs.push_back({x, 0});
        }
        c.card = uint32_t(c.vals.size());
        if (!c.card) continue;
        card_total += c.card;
        c.kind = c.card <= 4096 ? ARRAY : BITSET;
        const uint64_t run_bytes = 2 + 4ull * c.runs.size();
        if (run_bytes < (c.kind == ARRAY ? 2 + 2ull * c.card : 8192ull)) c.kind = RUN;
        cs.push_back(std::move(c));
    }
    const uint64_t size = cs.size();
    bool has_run = false;
    for (auto& c : cs) has_run = has_run || c.kind == RUN;
    uint64_t header = has_run ? 4 + (size + 7) / 8 + 4 * size + (size >= 4 ? 4 * size : 0) : 8 + 8 * size;
    uint64_t portable = header;
    for (auto& c : cs) portable += c.bytes();
    const uint64_t as_array = 4 * card_total + 4;
    auto put16 = [&](uint8_t* p, uint32_t v) { p[0] = uint8_t(v); p[1] = uint8_t(v >> 8); };
    auto put32 = [&](uint8_t* p, uint32_t v) { put16(p, v & 0xFFFF); put16(p + 2, v >> 16); };
    if (!(portable < as_array)) {  // CROARING_SERIALIZATION_ARRAY_UINT32
        const uint64_t total = 1 + as_array;
        if (total > cap) return total;
        out[0] = 1;
        put32(out + 1, uint32_t(card_total));
        uint64_t o = 5;
        for (auto& c : cs)
            for (uint16_t x : c.vals) { put32(out + o, (uint32_t(c.key) << 16) | x); o += 4; }
        return total;
    }
    const uint64_t total = 1 + portable;  // CROARING_SERIALIZATION_CONTAINER + portable format
    if (total > cap) return total;
    out[0] = 2;
    uint8_t* p = out + 1;
    uint64_t o = 0;
    if (has_run) {
        put32(p, 12347u | uint32_t((size - 1) << 16));
        o = 4;
        std::memset(p + o, 0, (size + 7) / 8);
        for (uint64_t k = 0; k < size; k++)
            if (cs[k].kind == RUN) p[o + k / 8] |= uint8_t(1u << (k % 8));
        o += (size + 7) / 8;
    } else {
        put32(p, 12346u);
        put32(p + 4, uint32_t(size));
        o = 8;
    }
    for (auto& c : cs) {
        put16(p + o, c.key);
        put16(p + o + 2, c.card - 1);
        o += 4;
    }
    if (!has_run || size >= 4) {
        uint32_t start = uint32_t(header);
        for (auto& c : cs) { put32(p + o, start); o += 4; start += uint32_t(c.bytes()); }
    }
    for (auto& c : cs) {
        if (c.kind == ARRAY) {
            for (uint16_t x : c.vals) { put16(p + o, x); o += 2; }
        } else if (c.kind == BITSET) {
            for (int w = 0; w < 1024; w++)
                for (int b = 0; b < 8; b++) p[o++] = uint8_t(c.words[w] >> (8 * b));
        } else {
            put16(p + o, uint32_t(c.runs.size()));
            o += 2;
            for (auto& r : c.runs) { put16(p + o, r.first); put16(p + o + 2, r.second); o += 4; }
        }
    }
    return total;
}

}  // extern "C"
