// eds-bwt_amd/tools/eds_common.h — EDS parsing and a reproducible RNG for the
// index writer (eds_transform) and the synthetic-input generator (edsbwt_gen).
//
// Parsing follows eds_to_fasta.cpp:55-153: '{' opens a segment and its first word,
// ',' opens the next word, an empty word (",," / "{," / ",}" or an explicit 'E',
// EMPTY_CHAR_EDS Parameters.h:33) becomes the single symbol 'Z' (EMPTY_CHAR,
// Parameters.h:34).  Inputs the reference chain cannot represent consistently are
// rejected with a message: "{}" (zero-length record), 'E' inside a word, bytes
// outside ('#','Z') (the terminator must be the smallest symbol and 'Z' the largest),
// and a last byte other than '}' (EDS-BWTransform.sh:11-14).
#pragma once
#include <cstdint>
#include <cstdio>
#include <stdexcept>
#include <string>
#include <vector>

namespace edsbwt_tools {

struct Eds {
    std::vector<uint8_t> text;      // words, each followed by '#'
    std::vector<uint64_t> wstart;   // text offset of each word
    std::vector<uint8_t> first;     // 1 if the word opens a segment
    uint64_t empty = 0, chars = 0;
};

inline std::vector<uint8_t> read_all(const std::string& path) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::runtime_error("Error: could not open file " + path);
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> b((size_t)n);
    if (n && std::fread(b.data(), 1, (size_t)n, f) != (size_t)n) { std::fclose(f); throw std::runtime_error("short read " + path); }
    std::fclose(f);
    return b;
}

inline Eds parse_eds(const std::vector<uint8_t>& s) {
    Eds E;
    const size_t n = s.size();
    if (!n) throw std::runtime_error("empty .eds");
    if (s[n - 1] != '}') throw std::runtime_error("ERROR: file .eds must end with }");
    if (s[0] != '{') throw std::runtime_error("Error: the string does not start with {.");
    E.text.reserve(n + n / 3);
    bool in_word = false;
    uint64_t wlen = 0;
    auto start_word = [&](int bit) {
        if (in_word) {
            if (!wlen) throw std::runtime_error("zero-length word ({} is not supported)");
            E.text.push_back('#');
        }
        E.wstart.push_back(E.text.size());
        E.first.push_back((uint8_t)bit);
        in_word = true;
        wlen = 0;
    };
    auto put = [&](uint8_t c) { E.text.push_back(c); wlen++; E.chars++; };
    start_word(1);
    if (n > 1 && s[1] == ',') { put('Z'); E.empty++; }
    for (size_t i = 1; i < n; i++) {
        const uint8_t c = s[i];
        const int next = i + 1 < n ? s[i + 1] : -1;
        if (c == '{') {
            start_word(1);
            if (next == ',') { put('Z'); E.empty++; }
        } else if (c == '}') {
        } else if (c == ',') {
            start_word(0);
            if (next == ',' || next == '}') { put('Z'); E.empty++; }
        } else if (c == 'E') {
            if (wlen || !(next == ',' || next == '}')) throw std::runtime_error("'E' inside a non-empty word at byte " + std::to_string(i));
            put('Z');
            E.empty++;
        } else {
            if (c <= '#' || c >= 'Z')
                throw std::runtime_error("Error: byte " + std::to_string(c) + " at " + std::to_string(i) + " is outside ('#','Z')");
            put(c);
        }
    }
    if (!wlen) throw std::runtime_error("zero-length word");
    E.text.push_back('#');
    return E;
}

// xoshiro256** seeded by splitmix64
struct Rng {
    uint64_t s[4];
    explicit Rng(uint64_t seed) {
        for (auto& x : s) {
            seed += 0x9e3779b97f4a7c15ull;
            uint64_t z = seed;
            z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
            z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
            x = z ^ (z >> 31);
        }
    }
    static uint64_t rotl(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
    uint64_t next() {
        const uint64_t r = rotl(s[1] * 5, 7) * 9, t = s[1] << 17;
        s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl(s[3], 45);
        return r;
    }
    uint64_t below(uint64_t n) { return (uint64_t)(((unsigned __int128)next() * n) >> 64); }
    uint64_t uni(uint64_t lo, uint64_t hi) { return lo + below(hi - lo + 1); }  // inclusive
    double unit() { return (double)(next() >> 11) * 0x1.0p-53; }
};

}  // namespace edsbwt_tools
