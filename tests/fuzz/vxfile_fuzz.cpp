// vxfile_fuzz.cpp — seeded mutation fuzzer of the Vortex file reader (vortex_amd/csrc/serde.cpp),
// built with -fsanitize=address,undefined (vortex_amd/csrc/Makefile target `sanitize`) and run by
// tests/test_sanitizers.py.  Test infrastructure: it links serde.cpp alone (host code, no HIP).
//
// What it checks (the reference's own defences are miri + a libfuzzer target,
// .github/workflows/ci.yml:58-72, fuzz/src/lib.rs:56-150; the reader restates
// vortex-serde/src/message_reader.rs:249-348 and layouts/read/footer.rs:140-187):
//   * the unmutated seed file opens, and every column's tree lies inside the file;
//   * for every mutation (bit flips, byte / word overwrites with boundary values, truncations,
//     insertions, deletions, block copies -- half of them aimed at the footer and the chunks'
//     message headers, where the flatbuffers live) every entry point returns a status, never
//     crashes, never reads outside the bytes it was given (ASan), never hits undefined
//     behaviour (UBSan, -fno-sanitize-recover), and every tree it does return has every buffer
//     inside the file (region = the whole file at file offset 0).
// Usage: vxfile_fuzz <seed.vortex> <iterations> <rng seed>   -> one JSON line of counts on stdout.
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <utility>
#include <vector>

#include "../../include/vortex_file.h"

namespace vxg {
// serde.cpp reports through the engine's error setter; the harness only needs the status
vxg_status set_error(vxg_status s, const std::string&) { return s; }
}  // namespace vxg

namespace {

struct Rng {
    uint64_t s;
    uint64_t next() {
        s ^= s << 13;
        s ^= s >> 7;
        s ^= s << 17;
        return s;
    }
    uint64_t below(uint64_t n) { return n ? next() % n : 0; }
};

struct Stats {
    uint64_t runs = 0, opened = 0, trees = 0, bad_trees = 0, nodes = 0;
    std::map<int, uint64_t> status;
};

// every buffer of the tree inside [0, len) (region NULL: pointers are file offsets)
bool tree_inside(const vxg_array* a, uint64_t len, int depth, Stats& st) {
    if (depth > 256) return false;
    st.nodes++;
    if (a->n_buffers && !a->buffers) return false;
    for (uint32_t i = 0; i < a->n_buffers; i++) {
        const uint64_t off = uint64_t(reinterpret_cast<uintptr_t>(a->buffers[i].ptr));
        const uint64_t n = a->buffers[i].len;
        if (off > len || n > len - off) return false;
    }
    if (a->n_children && !a->children) return false;
    for (uint32_t i = 0; i < a->n_children; i++)
        if (!tree_inside(&a->children[i], len, depth + 1, st)) return false;
    return true;
}

// Open + walk every entry point; returns false if a returned tree points outside the file.
bool run_one(const uint8_t* data, uint64_t len, Stats& st, bool must_open) {
    st.runs++;
    vxg_file* f = nullptr;
    vxg_status s = vxg_file_open(data, len, &f);
    if (s != VXG_OK) {
        st.status[int(s)]++;
        if (must_open) {
            std::fprintf(stderr, "seed file did not open: status %d\n", int(s));
            std::exit(2);
        }
        return true;
    }
    st.opened++;
    bool ok = true;
    uint64_t rows = 0;
    uint32_t ncols = 0;
    if (vxg_file_info(f, &rows, &ncols) == VXG_OK) {
        for (uint32_t c = 0; c < ncols && c < 64; c++) {
            vxg_file_column col{};
            if ((s = vxg_file_column_info(f, c, &col)) != VXG_OK) {
                st.status[int(s)]++;
                continue;
            }
            const uint32_t nch = col.n_chunks;
            for (uint32_t k = 0; k < nch && k < 8; k++) {
                vxg_file_chunk ch{};
                if ((s = vxg_file_chunk_info(f, c, k, &ch)) != VXG_OK) st.status[int(s)]++;
            }
            std::vector<uint64_t> offs(size_t(nch) + 1);
            if ((s = vxg_file_chunk_offsets(f, c, 0, nch, offs.data())) != VXG_OK) st.status[int(s)]++;
            // the whole column, then its first chunk alone
            const std::pair<uint32_t, uint32_t> ranges[2] = {{0, nch}, {0, nch ? 1u : 0u}};
            for (const auto& [b, e] : ranges) {
                const vxg_array* tree = nullptr;
                s = vxg_file_column_array(f, c, b, e, nullptr, 0, len, nullptr, &tree);
                if (s != VXG_OK) {
                    st.status[int(s)]++;
                    continue;
                }
                st.trees++;
                if (!tree || !tree_inside(tree, len, 0, st)) {
                    st.bad_trees++;
                    ok = false;
                }
            }
        }
    }
    vxg_file_close(f);
    return ok;
}

// Structural byte ranges of the seed: the last 64 KiB (footer, schema, postscript, EOF) and each
// chunk's message header [message_begin, buffers_begin).
std::vector<std::pair<uint64_t, uint64_t>> structure(const std::vector<uint8_t>& b) {
    std::vector<std::pair<uint64_t, uint64_t>> r;
    const uint64_t len = b.size();
    r.emplace_back(len > 65536 ? len - 65536 : 0, len);
    vxg_file* f = nullptr;
    if (vxg_file_open(b.data(), len, &f) != VXG_OK) return r;
    uint64_t rows = 0;
    uint32_t ncols = 0;
    vxg_file_info(f, &rows, &ncols);
    for (uint32_t c = 0; c < ncols; c++) {
        vxg_file_column col{};
        vxg_file_column_info(f, c, &col);
        for (uint32_t k = 0; k < col.n_chunks; k++) {
            vxg_file_chunk ch{};
            if (vxg_file_chunk_info(f, c, k, &ch) == VXG_OK && ch.buffers_begin > ch.message_begin)
                r.emplace_back(ch.message_begin, ch.buffers_begin);
        }
    }
    vxg_file_close(f);
    return r;
}

void mutate(std::vector<uint8_t>& m, Rng& rng, const std::vector<std::pair<uint64_t, uint64_t>>& hot) {
    static const uint64_t interesting[] = {0, 1, 0x7F, 0x80, 0xFF, 0x7FFF, 0xFFFF, 0x7FFFFFFF, 0xFFFFFFFF,
                                           0x80000000ull, ~0ull, 0x7FFFFFFFFFFFFFFFull, 64, 4096};
    const int ops = 1 + int(rng.below(4));
    for (int o = 0; o < ops && !m.empty(); o++) {
        uint64_t pos;
        if (rng.below(2) && !hot.empty()) {  // inside a structural range
            const auto& h = hot[rng.below(hot.size())];
            const uint64_t hi = h.second < m.size() ? h.second : m.size();
            pos = h.first < hi ? h.first + rng.below(hi - h.first) : rng.below(m.size());
        } else {
            pos = rng.below(m.size());
        }
        switch (rng.below(8)) {
        case 0: m[pos] ^= uint8_t(1u << rng.below(8)); break;                  // bit flip
        case 1: m[pos] = uint8_t(rng.next()); break;                            // random byte
        case 2: {                                                                // boundary word
            const uint64_t v = interesting[rng.below(sizeof(interesting) / 8)];
            const uint64_t w = uint64_t(1) << rng.below(4);                    // 1, 2, 4, 8 bytes
            for (uint64_t k = 0; k < w && pos + k < m.size(); k++) m[pos + k] = uint8_t(v >> (8 * k));
            break;
        }
        case 3: m.resize(pos); break;                                            // truncate
        case 4: {                                                                // insert bytes
            const uint64_t n = 1 + rng.below(16);
            m.insert(m.begin() + long(pos), size_t(n), uint8_t(rng.next()));
            break;
        }
        case 5: {                                                                // delete bytes
            const uint64_t n = 1 + rng.below(16);
            m.erase(m.begin() + long(pos), m.begin() + long(pos + n < m.size() ? pos + n : m.size()));
            break;
        }
        case 6: {                                                                // copy a block
            const uint64_t src = rng.below(m.size()), n = 1 + rng.below(64);
            for (uint64_t k = 0; k < n && src + k < m.size() && pos + k < m.size(); k++) m[pos + k] = m[src + k];
            break;
        }
        default: {                                                               // add a small delta
            m[pos] = uint8_t(m[pos] + uint8_t(1 + rng.below(4)) * (rng.below(2) ? 1 : 255));
            break;
        }
        }
    }
}

}  // namespace

int main(int argc, char** argv) {
    if (argc < 4) {
        std::fprintf(stderr, "usage: %s seed.vortex iterations rng_seed\n", argv[0]);
        return 2;
    }
    std::FILE* fp = std::fopen(argv[1], "rb");
    if (!fp) {
        std::perror(argv[1]);
        return 2;
    }
    std::vector<uint8_t> seed;
    uint8_t buf[1 << 16];
    size_t n;
    while ((n = std::fread(buf, 1, sizeof buf, fp)) > 0) seed.insert(seed.end(), buf, buf + n);
    std::fclose(fp);
    const uint64_t iters = std::strtoull(argv[2], nullptr, 10);
    Rng rng{std::strtoull(argv[3], nullptr, 10) * 0x9E3779B97F4A7C15ull | 1};
    Stats st;
    if (!run_one(seed.data(), seed.size(), st, true)) {
        std::fprintf(stderr, "seed file: a tree points outside the file\n");
        return 1;
    }
    const auto hot = structure(seed);
    uint64_t failures = 0;
    for (uint64_t i = 0; i < iters; i++) {
        std::vector<uint8_t> m = seed;
        mutate(m, rng, hot);
        // an exact-size heap copy, so ASan sees any read past the end of the mutated bytes
        uint8_t* exact = static_cast<uint8_t*>(std::malloc(m.size() ? m.size() : 1));
        if (!m.empty()) std::memcpy(exact, m.data(), m.size());
        if (!run_one(exact, m.size(), st, false)) failures++;
        std::free(exact);
    }
    std::printf("{\"iterations\": %llu, \"runs\": %llu, \"opened\": %llu, \"trees\": %llu, \"nodes\": %llu, "
                "\"bad_trees\": %llu, \"structural_ranges\": %zu, \"status\": {",
                (unsigned long long)iters, (unsigned long long)st.runs, (unsigned long long)st.opened,
                (unsigned long long)st.trees, (unsigned long long)st.nodes, (unsigned long long)st.bad_trees,
                hot.size());
    bool first = true;
    for (const auto& [k, v] : st.status) {
        std::printf("%s\"%d\": %llu", first ? "" : ", ", k, (unsigned long long)v);
        first = false;
    }
    std::printf("}}\n");
    return failures ? 1 : 0;
}
