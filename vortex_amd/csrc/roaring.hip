// roaring.hip — K16: RoaringBool canonicalize (croaring Native serialization -> LSB bit buffer).
//
// Reference: RoaringBoolArray::into_canonical = Bitmap::deserialize::<Native>(buffer).to_bitset()
// copied into a BooleanBuffer of len bits (encodings/roaring/src/boolean/mod.rs:69-72, 127-147);
// try_new requires cardinality <= len (:37-40).  croaring 2.1.1 (Cargo.lock) is not vendored, so
// its published format is restated (oracle/vx_oracle.c vxo_roaring_bool_decode is the CPU
// restatement; parity unpinned):
//   byte 0 = 1: u32 cardinality, then that many u32 values (any order);
//   byte 0 = 2: croaring's portable format at byte 1 — cookie 12346 + u32 size, or
//     12347 | (size - 1) << 16 + a bitset of run containers; then `size` (u16 key,
//     u16 cardinality - 1) pairs; then u32 container offsets (relative to byte 1) unless the
//     bitmap has runs and size < 4; containers: run = u16 n_runs + (u16 start, u16 length - 1)
//     pairs, cardinality <= 4096 = sorted u16 values, else 1024 little-endian u64 words.
// Like the reference's decode (try_from_parts does not re-run try_new's cardinality check),
// positions >= len are dropped.
//
// Layout on the GPU: one workgroup per 2^16-bit segment of the output (the span one container
// key covers).  Thread 0 parses the header and locates the segment's container (binary search
// of the keys); the workgroup builds the segment's 8 KiB of bits in LDS and ORs the non-zero
// words into the destination at its bit offset.  The u32-array form is spread over the same
// grid, one value per thread.  Every read is bounds-checked against the buffer length; a
// malformed serialization sets kErrRoaring (VXG_ERR_INVALID_SERDE).
#include "vxg_internal.hpp"

namespace vxg {

namespace {

constexpr int kRT = 256;
constexpr uint32_t kCookieRuns = 12347, kCookieNoRuns = 12346;

__device__ inline uint32_t rd16(const uint8_t* p) { return uint32_t(p[0]) | (uint32_t(p[1]) << 8); }
__device__ inline uint32_t rd32(const uint8_t* p) { return rd16(p) | (rd16(p + 2) << 16); }

// OR the 32 bits `word` (logical bits [q, q + 32)) into dst at bit position `bit` = off + q
__device__ inline void or_word(uint32_t* dst, uint64_t bit, uint32_t word) {
    const uint64_t w = bit >> 5;
    const unsigned sh = unsigned(bit & 31);
    atomicOr(dst + w, word << sh);
    if (sh) {
        const uint32_t hi = word >> (32 - sh);
        if (hi) atomicOr(dst + w + 1, hi);
    }
}

struct Seg {         // what thread 0 found for this workgroup's segment
    uint32_t fmt;    // 0 malformed, 1 u32 array, 2 portable
    uint32_t kind;   // 0 no container for this key, 1 array, 2 bitset, 3 run
    uint64_t pos;    // container bytes start (absolute offset in the buffer)
    uint32_t count;  // array cardinality / number of runs
};

__device__ void parse(const uint8_t* buf, uint64_t n, uint32_t key, Seg& s) {
    s.fmt = 0;
    s.kind = 0;
    s.count = 0;
    if (n < 1) return;
    if (buf[0] == 1) {
        if (n < 5) return;
        const uint32_t card = rd32(buf + 1);
        if (5 + 4ull * card > n) return;
        s.fmt = 1;
        s.count = card;
        return;
    }
    if (buf[0] != 2 || n < 5) return;
    const uint8_t* p = buf + 1;
    const uint64_t m = n - 1;
    const uint32_t cookie = rd32(p);
    uint64_t size, pos;
    uint64_t runbits = 0;  // offset of the run-container bitset in p (0: none)
    bool offsets;
    if ((cookie & 0xFFFF) == kCookieRuns) {
        size = (cookie >> 16) + 1ull;
        runbits = 4;
        pos = 4 + (size + 7) / 8;
        offsets = size >= 4;
    } else if (cookie == kCookieNoRuns) {
        if (m < 8) return;
        size = rd32(p + 4);
        pos = 8;
        offsets = true;
    } else {
        return;
    }
    if (size > 65536 || pos + 4 * size > m) return;
    const uint64_t desc = pos;
    pos += 4 * size;
    const uint64_t offs = pos;
    if (offsets) {
        if (pos + 4 * size > m) return;
        pos += 4 * size;
    }
    s.fmt = 2;
    // binary search for the key (keys strictly increasing; checked by the validation pass)
    uint64_t lo = 0, hi = size;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) / 2;
        if (rd16(p + desc + 4 * mid) < key) lo = mid + 1; else hi = mid;
    }
    if (lo == size || rd16(p + desc + 4 * lo) != key) return;  // empty segment
    const uint64_t k = lo;
    auto is_run = [&](uint64_t j) { return runbits && ((p[runbits + j / 8] >> (j % 8)) & 1); };
    auto card_of = [&](uint64_t j) { return rd16(p + desc + 4 * j + 2) + 1u; };
    uint64_t at;
    if (offsets) {
        at = rd32(p + offs + 4 * k);
    } else {  // walk the (at most three) containers before k
        at = pos;
        for (uint64_t j = 0; j < k; j++) {
            uint64_t b;
            if (is_run(j)) {
                if (at + 2 > m) { s.fmt = 0; return; }
                b = 2 + 4ull * rd16(p + at);
            } else {
                b = card_of(j) <= 4096 ? 2ull * card_of(j) : 8192;
            }
            at += b;
        }
    }
    uint64_t bytes;
    if (is_run(k)) {
        if (at + 2 > m) { s.fmt = 0; return; }
        s.kind = 3;
        s.count = rd16(p + at);
        bytes = 2 + 4ull * s.count;
    } else if (card_of(k) <= 4096) {
        s.kind = 1;
        s.count = card_of(k);
        bytes = 2ull * s.count;
    } else {
        s.kind = 2;
        s.count = card_of(k);
        bytes = 8192;
    }
    if (at + bytes > m) { s.fmt = 0; s.kind = 0; return; }
    s.pos = 1 + at;
}

__global__ __launch_bounds__(kRT) void roaring_bool_kernel(const uint8_t* __restrict__ buf, uint64_t n, uint64_t len,
                                                           uint32_t* __restrict__ dst, uint64_t off,
                                                           uint32_t* __restrict__ err) {
    __shared__ Seg s;
    __shared__ uint32_t s_bits[2048];
    __shared__ uint32_t s_bad;
    const unsigned tid = threadIdx.x;
    const uint32_t key = blockIdx.x;
    if (tid == 0) {
        parse(buf, n, key, s);
        s_bad = s.fmt == 0;
    }
    for (unsigned w = tid; w < 2048; w += kRT) s_bits[w] = 0;
    __syncthreads();
    if (s.fmt == 0) {
        if (tid == 0) __hip_atomic_fetch_or(err, kErrRoaring, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    if (s.fmt == 1) {  // u32 values, one per thread over the whole grid
        for (uint64_t i = uint64_t(key) * kRT + tid; i < s.count; i += uint64_t(gridDim.x) * kRT) {
            const uint64_t v = rd32(buf + 5 + 4 * i);
            if (v < len) {
                const uint64_t b = off + v;
                atomicOr(dst + (b >> 5), 1u << (b & 31));
            }
        }
        return;
    }
    if (key == 0) {  // validation pass: keys strictly increasing (croaring's deserialize_safe)
        const uint8_t* p = buf + 1;
        const uint32_t cookie = rd32(p);
        const bool runs = (cookie & 0xFFFF) == kCookieRuns;
        const uint64_t size = runs ? (cookie >> 16) + 1ull : rd32(p + 4);
        const uint64_t desc = runs ? 4 + (size + 7) / 8 : 8;
        bool bad = false;
        for (uint64_t j = tid + 1; j < size; j += kRT)
            bad |= rd16(p + desc + 4 * j) <= rd16(p + desc + 4 * (j - 1));
        if (bad) s_bad = 1;  // benign race: every writer stores 1
    }
    const uint8_t* c = buf + s.pos;
    if (s.kind == 1) {
        for (unsigned i = tid; i < s.count; i += kRT) {
            const uint32_t x = rd16(c + 2 * i);
            atomicOr(&s_bits[x >> 5], 1u << (x & 31));
        }
    } else if (s.kind == 2) {
        const bool al = (reinterpret_cast<uintptr_t>(c) & 3) == 0;
        for (unsigned w = tid; w < 2048; w += kRT) s_bits[w] = al ? reinterpret_cast<const uint32_t*>(c)[w] : rd32(c + 4 * w);
    } else if (s.kind == 3) {
        for (unsigned r = tid; r < s.count; r += kRT) {
            const uint32_t st = rd16(c + 2 + 4 * r), ln = rd16(c + 4 + 4 * r);
            if (st + ln > 65535) { s_bad = 1; continue; }
            const uint32_t e = st + ln;  // inclusive
            const uint32_t w0 = st >> 5, w1 = e >> 5;
            for (uint32_t w = w0; w <= w1; w++) {
                uint32_t m = ~0u;
                if (w == w0) m &= ~0u << (st & 31);
                if (w == w1) m &= ~0u >> (31 - (e & 31));
                atomicOr(&s_bits[w], m);
            }
        }
    }
    __syncthreads();
    if (s_bad) {
        if (tid == 0) __hip_atomic_fetch_or(err, kErrRoaring, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return;
    }
    const uint64_t base = uint64_t(key) << 16;
    for (unsigned w = tid; w < 2048; w += kRT) {
        const uint64_t q = base + 32ull * w;
        if (q >= len) break;
        uint32_t word = s_bits[w];
        if (len - q < 32) word &= (1u << (len - q)) - 1u;
        if (word) or_word(dst, off + q, word);
    }
}

}  // namespace

vxg_status launch_roaring_bool(const uint8_t* buf, uint64_t n, uint64_t len, void* bits, uint64_t off, uint32_t* err,
                               hipStream_t s) {
    if (len == 0) return VXG_OK;
    const uint64_t segs = (len + 65535) >> 16;  // <= 65536 for any u32-addressable bitmap
    if (segs > 65536) return set_error(VXG_ERR_INVALID_ARGUMENT, "RoaringBool longer than 2^32");
    hipLaunchKernelGGL(roaring_bool_kernel, dim3(unsigned(segs)), dim3(kRT), 0, s, buf, n, len,
                       static_cast<uint32_t*>(bits), off, err);
    return hip_check(hipGetLastError(), "roaring_bool_kernel");
}

}  // namespace vxg
