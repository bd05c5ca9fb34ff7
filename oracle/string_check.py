"""Test infrastructure (checker only): a pure-Python restatement of the reference's
stringCheck (stringCheck.cpp:11-106), written straight from its loop, to check
eds-bwt_amd/tools/string_check.cpp byte for byte.

Returns (output bytes, exit code).  The reference's `next` is a char, so a 0xFF byte reads
as EOF (:50-51).  Where the reference has no defined behaviour, this returns what the tool
does: an empty input gives b"" (exit 0), an unclosed '<' gives exit 1."""

EMPTY_CHAR = ord("Z")  # Parameters.h:34
EOF_ = -1


def string_check(data: bytes):
    out = bytearray()
    n = len(data)

    def peek(i):
        if i >= n or data[i] == 0xFF:
            return EOF_
        return data[i]

    if n == 0:
        return bytes(out), 0
    cur = data[0]                       # :28
    if cur == EMPTY_CHAR:               # :29, :37-40
        return bytes(out), 1
    if cur == ord("{"):
        out.append(cur)
    else:
        out += b"{" + bytes([cur])
    i = 1
    while i < n:                        # :43
        cur = data[i]
        if cur == EMPTY_CHAR:           # :45-48
            return bytes(out), 1
        nxt = peek(i + 1)               # :50
        if cur == ord("}") and nxt != ord("{") and nxt != EOF_:      # :51
            out += b"}{"
        elif cur != ord("}") and nxt == ord("{"):                    # :54
            out += bytes([cur]) + b"}"
        elif cur == ord("<"):                                        # :57-65
            j = i + 1
            while j < n and data[j] != ord(">"):
                j += 1
            if j >= n:
                return bytes(out), 1
            i = j
            if peek(i + 1) == ord("{"):
                out += b"}"
        elif nxt == EOF_ and cur != ord("}"):                        # :67
            out += bytes([cur]) + b"}"
        else:                                                        # :70
            out.append(cur)
        i += 1
    return bytes(out), 0
