// eds-bwt_amd/tools/string_check.cpp — `stringCheck <input> <output>`: normalises an
// elastic-degenerate string before the index writer (eds_transform), as the reference's
// stringCheck.cpp:11-106 does: curly brackets around every solid stretch, "<...>" comments
// dropped, and a hard error on the symbol the index uses for the empty word (EMPTY_CHAR 'Z',
// Parameters.h:34).  The output goes to "<output>.eds".
//
// The rules, one input byte `cur` at a time with `next` the byte after it (EOF past the end):
//   first byte: 'Z' -> error; '{' -> "{"; else "{" cur                          (:28-40)
//   then, for each byte, first rule that applies:                               (:43-73)
//     'Z'                                   -> error
//     cur == '}' && next != '{' && next != EOF -> "}{"
//     cur != '}' && next == '{'             -> cur "}"
//     cur == '<'                            -> skip through the next '>'; "}" if then next == '{'
//     next == EOF && cur != '}'             -> cur "}"
//     otherwise                             -> cur
// Kept as the reference behaves: a 0xFF byte compares equal to EOF in the `next` tests (the
// reference keeps `next` in a char), a first byte '<' is copied, a trailing '\n' gets a '}'
// after it.  Differences, where the reference has no defined behaviour: an empty input gives an
// empty output (the reference reads an uninitialised char), and a '<' with no closing '>'
// is an error (the reference loops forever on the failed get()).
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

static const char kEmptyChar = 'Z';  // EMPTY_CHAR, Parameters.h:34

static void empty_char_error() {
    std::fprintf(stderr,
                 "\n\nError: the input contains character %c, which is used by this tool to represent an empty string. Please change EMPTY"
                 "_CHAR in Parameters.h or change the character in your input.\n\n\n",
                 kEmptyChar);
    std::exit(1);
}

int main(int argc, char** argv) {
    if (argc != 3) {
        std::fprintf(stderr, "usage: %s inputoutput\n", argv[0]);
        std::fprintf(stderr, "input is the full filename, output will have \".eds\" appended.\n");
        return 1;
    }
    const std::string in_name = argv[1], out_name = std::string(argv[2]) + ".eds";
    std::printf("stringCheck on %s, output %s\n", in_name.c_str(), out_name.c_str());
    std::fflush(stdout);
    FILE* fi = std::fopen(in_name.c_str(), "rb");
    FILE* fo = fi ? std::fopen(out_name.c_str(), "wb") : nullptr;
    if (!fi || !fo) {
        std::fprintf(stderr, "Error: cannot open file %s or file %s\n", in_name.c_str(), out_name.c_str());
        return 1;
    }
    std::vector<unsigned char> b;
    {
        unsigned char buf[1 << 16];
        size_t n;
        while ((n = std::fread(buf, 1, sizeof buf, fi)) > 0) b.insert(b.end(), buf, buf + n);
    }
    std::fclose(fi);
    std::string out;
    out.reserve(b.size() + b.size() / 8 + 16);
    const size_t n = b.size();
    // `next` as the reference sees it: a char, so byte 0xFF reads as EOF
    auto next_is_eof = [&](size_t i) { return i >= n || b[i] == 0xFF; };
    auto next_is = [&](size_t i, char c) { return i < n && b[i] == (unsigned char)c; };
    if (n) {
        const char c0 = (char)b[0];
        if (c0 == kEmptyChar) empty_char_error();
        if (c0 != '{') out.push_back('{');
        out.push_back(c0);
    }
    for (size_t i = 1; i < n; i++) {
        const char cur = (char)b[i];
        if (cur == kEmptyChar) {
            std::fwrite(out.data(), 1, out.size(), fo);
            std::fclose(fo);
            empty_char_error();
        }
        if (cur == '}' && !next_is(i + 1, '{') && !next_is_eof(i + 1)) {
            out += "}{";
        } else if (cur != '}' && next_is(i + 1, '{')) {
            out.push_back(cur);
            out.push_back('}');
        } else if (cur == '<') {
            size_t j = i + 1;
            while (j < n && b[j] != '>') j++;
            if (j >= n) {
                std::fwrite(out.data(), 1, out.size(), fo);
                std::fclose(fo);
                std::fprintf(stderr, "Error: '<' at byte %zu of %s has no closing '>'\n", i, in_name.c_str());
                return 1;
            }
            i = j;  // the '>' is consumed with the comment
            if (next_is(i + 1, '{')) out.push_back('}');
        } else if (next_is_eof(i + 1) && cur != '}') {
            out.push_back(cur);
            out.push_back('}');
        } else {
            out.push_back(cur);
        }
    }
    std::fwrite(out.data(), 1, out.size(), fo);
    std::fclose(fo);
    std::printf("Done.\n");
    return 0;
}
