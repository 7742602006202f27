// rx_flows.h — host side of the flow tables: the control-block registry and
// the host image of every device table (layouts in rx_common.h), kept
// incrementally so that a connection opened or closed between bursts costs
// O(1) host work and a handful of slot writes on the device, not a rebuild.
//
// Reference semantics kept:
//   - get_hostinfo_fromip_port (common.c:97-108) and pass 1 of
//     tcp_stream_search (common.c:31-55) return the FIRST match of a
//     head-inserted list (LL_ADD, common.h:43-49), i.e. the NEWEST control
//     block with the key.  Every block carries a creation sequence number;
//     blocks sharing a key form a chain newest -> oldest, and the table slot
//     of the key holds the chain's head.  Removing the head exposes the next
//     older block (the list walk would find it next).
//   - pass 2 of tcp_stream_search: the newest LISTEN block on the dst port,
//     dst ip ignored (direct table indexed by the raw port).
//   - tcbs are created on SYN (tcp.c:50-52, LL_ADD) and freed on the last ACK
//     and on close (tcp.c:321, common.c:620,660): rx_flowset::add / remove.
//
// Ids are stable: a block keeps its flow id for life (verdict flow_id, count
// index), freed ids are reused, newest first.  Tables are linear-probed with
// backward-shift deletion (no tombstones: the device probes stop at the first
// empty slot) and a per-context hash seed (rxg_open draws it at random), so
// remote peers, who choose the tcb keys on every SYN (tcp.c:50), cannot aim
// at probe clusters; a probe sequence longer than RX_PROBE_CAP reseeds.
#pragma once

#include <stdint.h>

#include <algorithm>
#include <unordered_map>
#include <vector>

#include "rx_common.h"

#define RX_PROBE_CAP 48u // longest probe sequence accepted before a reseed

struct rx_block {
    uint32_t a = 0, b = 0, c = 0; // key (rx_common.h): UDP (dip, dport, 17), TCP (sip, dip, ports)
    uint32_t status = 0;          // tcb status (LISTEN = 1); UDP: the socket's protocol
    uint64_t seq = 0;             // creation order: the higher, the newer
    uint32_t older = RXG_FLOW_NONE; // next older live block with the same key
    bool live = false;
    bool keyed = false;           // in the exact-key table (UDP: protocol 17 only)
};

// One exact-key table (UDP or TCP): the slot array as the device holds it.
struct rx_slot_table {
    std::vector<uint4> slots; // ns + RX_FT_MIRROR (the mirror repeats slots 0..)
    uint32_t mask = 0, probe = 1, seed = 0, used = 0;
    std::vector<uint32_t> dirty; // slots written since the last upload
    bool all_dirty = true;       // the whole array must be uploaded

    uint32_t ns() const { return mask + 1; }
    uint32_t home(uint32_t a, uint32_t b, uint32_t c) const { return rx_hash3s(seed, a, b, c) & mask; }

    void reset(uint32_t nslots, uint32_t sd) {
        slots.assign((size_t)nslots + RX_FT_MIRROR, make_uint4(0, 0, 0, RX_SLOT_EMPTY));
        mask = nslots - 1;
        probe = 1;
        seed = sd;
        used = 0;
        dirty.clear();
        all_dirty = true;
    }
    void touch(uint32_t i) {
        if (i < RX_FT_MIRROR) slots[ns() + i] = slots[i];
        if (all_dirty) return;
        dirty.push_back(i);
        if (i < RX_FT_MIRROR) dirty.push_back(ns() + i);
    }
    uint32_t find(uint32_t a, uint32_t b, uint32_t c) const {
        uint32_t i = home(a, b, c);
        for (;;) {
            const uint4 &s = slots[i];
            if (s.w == RX_SLOT_EMPTY) return ~0u;
            if (s.x == a && s.y == b && s.z == c) return i;
            i = (i + 1) & mask;
        }
    }
    uint32_t lookup(uint32_t a, uint32_t b, uint32_t c) const {
        const uint32_t i = find(a, b, c);
        return i == ~0u ? RXG_FLOW_NONE : slots[i].w;
    }
    // key absent: the first empty slot of its probe sequence; false when the
    // sequence exceeds RX_PROBE_CAP (the slot is written anyway; the caller
    // rebuilds with another seed)
    bool insert(uint32_t a, uint32_t b, uint32_t c, uint32_t w) {
        uint32_t i = home(a, b, c), d = 0;
        while (slots[i].w != RX_SLOT_EMPTY) i = (i + 1) & mask, ++d;
        slots[i] = make_uint4(a, b, c, w);
        touch(i);
        ++used;
        probe = std::max(probe, d + 1);
        return d + 1 <= RX_PROBE_CAP;
    }
    void set(uint32_t i, uint32_t w) {
        slots[i].w = w;
        touch(i);
    }
    // backward-shift deletion (Knuth 6.4 algorithm R): later members of the
    // cluster whose home does not lie cyclically in (i, j] move back into the
    // hole, so no probe sequence crosses an empty slot
    void erase(uint32_t i) {
        uint32_t j = i;
        for (;;) {
            j = (j + 1) & mask;
            const uint4 &s = slots[j];
            if (s.w == RX_SLOT_EMPTY) break;
            const uint32_t k = home(s.x, s.y, s.z);
            const bool stays = i <= j ? (i < k && k <= j) : (i < k || k <= j);
            if (stays) continue;
            slots[i] = s;
            touch(i);
            i = j;
        }
        slots[i] = make_uint4(0, 0, 0, RX_SLOT_EMPTY);
        touch(i);
        --used;
    }
};

// The control blocks of one protocol and their exact-key table.
struct rx_registry {
    std::vector<rx_block> blk; // by flow id
    std::vector<uint32_t> free_ids;
    uint32_t live = 0;
    uint64_t seq_next = 0;
    rx_slot_table tab;

    uint32_t id_space() const { return (uint32_t)blk.size(); }
    uint32_t alloc_id() {
        if (!free_ids.empty()) {
            const uint32_t id = free_ids.back();
            free_ids.pop_back();
            return id;
        }
        blk.emplace_back();
        return (uint32_t)blk.size() - 1;
    }
    // link block id into its key's chain (by seq) and the table; false = probe cap hit
    bool link(uint32_t id) {
        rx_block &x = blk[id];
        const uint32_t i = tab.find(x.a, x.b, x.c);
        if (i == ~0u) {
            x.older = RXG_FLOW_NONE;
            return tab.insert(x.a, x.b, x.c, id);
        }
        const uint32_t head = tab.slots[i].w;
        if (x.seq > blk[head].seq) {
            x.older = head;
            tab.set(i, id);
            return true;
        }
        uint32_t p = head;
        while (blk[p].older != RXG_FLOW_NONE && blk[blk[p].older].seq > x.seq) p = blk[p].older;
        x.older = blk[p].older;
        blk[p].older = id;
        return true;
    }
    void unlink(uint32_t id) {
        rx_block &x = blk[id];
        const uint32_t i = tab.find(x.a, x.b, x.c);
        if (i == ~0u) return; // (not reached: a keyed block is always in its chain)
        const uint32_t head = tab.slots[i].w;
        if (head == id) {
            if (x.older != RXG_FLOW_NONE)
                tab.set(i, x.older);
            else
                tab.erase(i);
        } else {
            uint32_t p = head;
            while (p != RXG_FLOW_NONE && blk[p].older != id) p = blk[p].older;
            if (p != RXG_FLOW_NONE) blk[p].older = x.older;
        }
        x.older = RXG_FLOW_NONE;
    }
    // every keyed live block into a fresh table of nslots (chains kept: they
    // do not depend on the slot layout); false = probe cap hit
    bool rebuild(uint32_t nslots, uint32_t seed) {
        tab.reset(nslots, seed);
        bool ok = true;
        for (uint32_t id = 0; id < blk.size(); ++id) {
            const rx_block &x = blk[id];
            if (!x.live || !x.keyed) continue;
            const uint32_t i = tab.find(x.a, x.b, x.c);
            if (i == ~0u)
                ok &= tab.insert(x.a, x.b, x.c, id);
            else if (x.seq > blk[tab.slots[i].w].seq)
                tab.slots[i].w = id;
        }
        for (uint32_t k = 0; k < RX_FT_MIRROR; ++k) tab.slots[tab.ns() + k] = tab.slots[k];
        return ok;
    }
};

// Everything the device probes, as host images plus what changed since the
// last upload: the two exact-key tables, the listener table, the UDP port
// table (and its per-port count of sockets on other addresses), the compact
// UDP table and port window (small: rebuilt whole when the sockets change).
struct rx_flowset {
    rx_registry udp, tcp;
    uint32_t seed = 0x9E3779B9u;
    uint32_t load_log2 = RX_FT_LOAD_LOG2;
    bool port_table = true;  // !RXG_TT_NO_UDP_PORT
    // listeners: newest LISTEN block per raw dport
    std::vector<uint32_t> listen = std::vector<uint32_t>(65536, RXG_FLOW_NONE);
    std::unordered_map<uint32_t, std::vector<uint32_t>> listeners; // raw dport -> LISTEN ids
    std::vector<uint32_t> listen_dirty;
    bool listen_all_dirty = true;
    // UDP port table (rx_udp_port_decide): empty when not built
    std::vector<uint32_t> port;
    std::vector<uint32_t> port_other; // sockets on the port bound to another address
    uint32_t udp_dip = 0, on_dip = 0; // the table's address, live keyed sockets on it
    std::vector<uint32_t> port_dirty;
    bool port_all_dirty = true;
    // compact UDP table + port window (rx_common.h), derived
    std::vector<uint2> udpc;
    uint32_t udpc_probe = 0;
    uint32_t udpc_other = 0; // compact keys whose address is not udp_dip
    std::vector<uint16_t> udpw;
    uint32_t udpw_lo = 0;
    bool small_dirty = true;
    uint32_t rebuilds = 0; // full table rebuilds (growth, reseeds), for tests

    static uint32_t slots_for(uint32_t keys, uint32_t load_log2) {
        uint64_t ns = 16;
        while (ns < ((uint64_t)keys << load_log2)) ns <<= 1;
        return (uint32_t)ns;
    }

    // ---- listeners
    void listen_recompute(uint32_t dport) {
        uint32_t best = RXG_FLOW_NONE;
        auto it = listeners.find(dport);
        if (it != listeners.end())
            for (uint32_t id : it->second)
                if (best == RXG_FLOW_NONE || tcp.blk[id].seq > tcp.blk[best].seq) best = id;
        if (listen[dport] != best) {
            listen[dport] = best;
            if (!listen_all_dirty) listen_dirty.push_back(dport);
        }
    }
    void listen_add(uint32_t id) {
        const uint32_t dp = tcp.blk[id].c >> 16;
        listeners[dp].push_back(id);
        listen_recompute(dp);
    }
    void listen_del(uint32_t id) {
        const uint32_t dp = tcp.blk[id].c >> 16;
        auto it = listeners.find(dp);
        if (it == listeners.end()) return;
        std::vector<uint32_t> &v = it->second;
        v.erase(std::remove(v.begin(), v.end(), id), v.end());
        if (v.empty()) listeners.erase(it);
        listen_recompute(dp);
    }

    // ---- UDP port table
    void port_recompute(uint32_t p) {
        if (port.empty()) return;
        const uint32_t f = udp.tab.lookup(udp_dip, p, 17u);
        const uint32_t e = (port_other[p] ? RX_PORT_HASHED : 0u) | (f == RXG_FLOW_NONE ? RX_PORT_NONE : f);
        if (port[p] != e) {
            port[p] = e;
            if (!port_all_dirty) port_dirty.push_back(p);
        }
    }
    // the whole port table for the address most live sockets are bound to
    void port_rebuild() {
        port.clear();
        port_other.clear();
        on_dip = 0;
        port_all_dirty = true;
        port_dirty.clear();
        if (!port_table || udp.live == 0) return;
        std::unordered_map<uint32_t, uint32_t> dips;
        for (const rx_block &x : udp.blk)
            if (x.live && x.keyed) ++dips[x.a];
        uint32_t best = 0;
        udp_dip = 0;
        for (const auto &d : dips)
            if (d.second > best || (d.second == best && d.first < udp_dip)) best = d.second, udp_dip = d.first;
        port.assign(65536, RX_PORT_NONE);
        port_other.assign(65536, 0);
        for (const rx_block &x : udp.blk) {
            if (!x.live || !x.keyed) continue;
            if (x.a == udp_dip)
                ++on_dip;
            else
                ++port_other[x.b & 0xFFFFu];
        }
        for (uint32_t p = 0; p < 65536; ++p) port_recompute(p);
    }
    void port_track(const rx_block &x, int delta) { // a keyed socket came (+1) or went (-1)
        if (port.empty()) return;
        if (x.a == udp_dip)
            on_dip += delta;
        else
            port_other[x.b & 0xFFFFu] += delta;
        port_recompute(x.b & 0xFFFFu);
    }

    // ---- compact UDP table + port window (lane kernel, <= 1024 sockets)
    void small_rebuild() {
        small_dirty = true;
        udpc.clear();
        udpc_probe = 0;
        udpc_other = 0;
        udpw.clear();
        udpw_lo = 0;
        // flow ids are stored in 16 bits (compact slot) and as u16 != 0xFFFF (window)
        if (udp.live == 0 || udp.live > RX_UDPC_MAX_FLOWS || udp.id_space() >= 0xFFFFu) return;
        uint32_t ns = 16;
        while (ns < 2 * udp.live) ns <<= 1;
        udpc.assign(ns, make_uint2(0, 0xFFFFFFFFu));
        const uint32_t mask = ns - 1;
        for (uint32_t j = 0; j < udp.tab.ns(); ++j) {
            const uint4 &sl = udp.tab.slots[j];
            if (sl.w == RX_SLOT_EMPTY) continue; // key (dip, dport, 17) -> newest flow
            uint32_t i = rx_hash3s(seed, sl.x, sl.y, sl.z) & mask, d = 0;
            while (udpc[i].y != 0xFFFFFFFFu) i = (i + 1) & mask, ++d;
            udpc[i] = make_uint2(sl.x, (sl.y & 0xFFFFu) | (sl.w << 16));
            udpc_probe = std::max(udpc_probe, d + 1);
            if (sl.x != udp_dip) ++udpc_other;
        }
        if (port.empty()) return;
        uint32_t mn = 65536, mx = 0;
        for (uint32_t r = 0; r < 65536; ++r)
            if ((port[r] & RX_PORT_NONE) != RX_PORT_NONE) {
                const uint32_t h = rx_bswap16(r);
                mn = std::min(mn, h);
                mx = std::max(mx, h);
            }
        if (mn > mx || mx - mn + 1 > RX_UDPW_MAX_PORTS) return;
        udpw.assign(mx - mn + 1, 0xFFFFu);
        for (uint32_t h = mn; h <= mx; ++h) {
            const uint32_t f = port[rx_bswap16(h)] & RX_PORT_NONE;
            if (f != RX_PORT_NONE) udpw[h - mn] = (uint16_t)f;
        }
        udpw_lo = mn;
    }

    // ---- whole-set operations
    // both exact-key tables from scratch (sized for the live keys at the load
    // factor, reseeded until no probe sequence exceeds RX_PROBE_CAP), then the
    // derived tables
    // extra_u / extra_t: keys about to be added (sizes the tables for them)
    void rebuild_all(uint32_t (*next_seed)(uint32_t), uint32_t extra_u = 0, uint32_t extra_t = 0) {
        uint32_t ku = extra_u, kt = extra_t;
        for (const rx_block &x : udp.blk) ku += x.live && x.keyed;
        for (const rx_block &x : tcp.blk) kt += x.live && x.keyed;
        uint32_t nu = slots_for(ku, load_log2), nt = slots_for(kt, load_log2);
        for (int tries = 1;; ++tries) {
            const bool ou = udp.rebuild(nu, seed), ot = tcp.rebuild(nt, seed);
            if (ou && ot) break;
            seed = next_seed(seed); // (one seed for every table: a reseed rebuilds both)
            if (tries % 4 == 0) nu <<= !ou, nt <<= !ot;
        }
        ++rebuilds;
        listen_all_dirty = true;
        listen_dirty.clear();
        port_rebuild();
        small_rebuild();
    }
    void clear() {
        udp = rx_registry();
        tcp = rx_registry();
        listen.assign(65536, RXG_FLOW_NONE);
        listeners.clear();
    }
    // after an insert that hit the probe cap, or a table past load 1/2
    bool needs_rebuild(const rx_registry &r, bool cap_hit) const {
        return cap_hit || (uint64_t)r.tab.used * 2 > r.tab.ns();
    }
};
