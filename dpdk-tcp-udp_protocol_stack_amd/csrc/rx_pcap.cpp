// rx_pcap.cpp — host ingest for librxgpu: classic pcap files (LINKTYPE_ETHERNET)
// read into, and written from, the packed burst layout of include/rxgpu.h.
//
// This is the stand-in for the reference's NIC front end (rte_eth_rx_burst
// into the in-ring, netfamily.c:438-440, dequeued 32 at a time at :147): a
// capture file is mapped once and consumed burst by burst, each frame copied
// to a (1 << off_unit_log2)-aligned start in the caller's (ideally pinned)
// buffer with zero fill up to the next 16-B boundary, as rxg_classify* expect.
#include <errno.h>
#include <fcntl.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <new>

#include "../../include/rxgpu.h"

struct rxg_pcap {
    const uint8_t *map = nullptr;
    size_t size = 0;
    size_t pos = 24; // first record header
    bool swap = false;
    uint64_t frames = 0; // frames consumed so far
};

static uint32_t rd32(const uint8_t *p, bool swap) {
    uint32_t v;
    memcpy(&v, p, 4);
    return swap ? __builtin_bswap32(v) : v;
}

extern "C" {

int rxg_pcap_open(rxg_pcap **out, const char *path) {
    if (!out || !path) return RXG_EINVAL;
    *out = nullptr;
    const int fd = open(path, O_RDONLY);
    if (fd < 0) return RXG_EINVAL;
    struct stat st;
    if (fstat(fd, &st) != 0 || st.st_size < 24) {
        close(fd);
        return RXG_EINVAL;
    }
    void *m = mmap(nullptr, (size_t)st.st_size, PROT_READ, MAP_PRIVATE, fd, 0);
    close(fd);
    if (m == MAP_FAILED) return RXG_ENOMEM;
    const uint8_t *b = (const uint8_t *)m;
    uint32_t magic;
    memcpy(&magic, b, 4);
    bool swap;
    if (magic == 0xA1B2C3D4u || magic == 0xA1B23C4Du) // microsecond / nanosecond stamps
        swap = false;
    else if (magic == 0xD4C3B2A1u || magic == 0x4D3CB2A1u)
        swap = true;
    else {
        munmap(m, (size_t)st.st_size);
        return RXG_EINVAL;
    }
    if (rd32(b + 20, swap) != 1u) { // LINKTYPE_ETHERNET only (the stack's rx port)
        munmap(m, (size_t)st.st_size);
        return RXG_EINVAL;
    }
    rxg_pcap *p = new (std::nothrow) rxg_pcap();
    if (!p) {
        munmap(m, (size_t)st.st_size);
        return RXG_ENOMEM;
    }
    p->map = b;
    p->size = (size_t)st.st_size;
    p->swap = swap;
    *out = p;
    return RXG_OK;
}

void rxg_pcap_close(rxg_pcap *p) {
    if (!p) return;
    if (p->map) munmap((void *)p->map, p->size);
    delete p;
}

int rxg_pcap_rewind(rxg_pcap *p) {
    if (!p) return RXG_EINVAL;
    p->pos = 24;
    p->frames = 0;
    return RXG_OK;
}

int rxg_pcap_read_burst(rxg_pcap *p, uint8_t *pkts, uint64_t cap_bytes, uint32_t *off,
                        uint16_t *len, uint32_t max_frames, uint32_t off_unit_log2, uint32_t *n,
                        uint64_t *span) {
    if (n) *n = 0;
    if (span) *span = 0;
    if (!p || !pkts || !off || !len || !n) return RXG_EINVAL;
    if (off_unit_log2 < 4 || off_unit_log2 > 16) return RXG_EINVAL;
    const uint64_t unit = 1ull << off_unit_log2;
    uint64_t pos = 0;
    uint32_t k = 0;
    while (k < max_frames && p->pos + 16 <= p->size) {
        const uint8_t *rh = p->map + p->pos;
        const uint32_t incl = rd32(rh + 8, p->swap);
        if (incl > 65535u) return RXG_ERANGE;           // verdict lengths are u16
        if (p->pos + 16 + incl > p->size) return RXG_EINVAL; // truncated record
        const uint64_t step = incl ? (incl + unit - 1) & ~(unit - 1) : unit;
        if ((pos >> off_unit_log2) > 0xFFFFFFFFull) return RXG_ERANGE;
        if (pos + step > cap_bytes) {
            if (k == 0) return RXG_ERANGE; // one frame does not fit the buffer
            break;
        }
        memcpy(pkts + pos, rh + 16, incl);
        const uint64_t end16 = (incl + 15) & ~15ull;
        if (end16 > incl) memset(pkts + pos + incl, 0, end16 - incl);
        off[k] = (uint32_t)(pos >> off_unit_log2);
        len[k] = (uint16_t)incl;
        pos += step;
        p->pos += 16 + incl;
        ++k;
    }
    p->frames += k;
    *n = k;
    if (span) *span = pos;
    return RXG_OK;
}

int rxg_pcap_write(const char *path, const uint8_t *pkts, const uint32_t *off, const uint16_t *len,
                   uint32_t n, uint32_t off_unit_log2) {
    if (!path || (n && (!pkts || !off || !len))) return RXG_EINVAL;
    if (off_unit_log2 > 16) return RXG_EINVAL;
    FILE *f = fopen(path, "wb");
    if (!f) return RXG_EINVAL;
    const uint32_t gh[6] = {0xA1B2C3D4u, 2u | (4u << 16), 0u, 0u, 65535u, 1u};
    bool ok = fwrite(gh, 4, 6, f) == 6;
    for (uint32_t i = 0; ok && i < n; ++i) {
        const uint32_t rh[4] = {i / 1000000u, i % 1000000u, len[i], len[i]};
        ok = fwrite(rh, 4, 4, f) == 4 &&
             fwrite(pkts + ((uint64_t)off[i] << off_unit_log2), 1, len[i], f) == len[i];
    }
    ok = (fclose(f) == 0) && ok;
    return ok ? RXG_OK : RXG_EINVAL;
}

} // extern "C"
