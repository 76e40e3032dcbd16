// philox.h — Philox4x32-10 counter-based RNG, host + device.
//
// Every random choice the reference makes with the global math/rand source
// (shufflePeers/shuffleStrings gossipsub.go:1954-1973, AddPromise
// gossip_tracer.go:53) is replaced by a Philox draw keyed on
// (seed) and countered on (tick, observer, topic|purpose, item), so a choice is
// a pure function of its coordinates: the GPU and the CPU oracle make the same
// choice regardless of thread schedule.
#pragma once
#include <stdint.h>

#if defined(__HIPCC__)
#define GSIM_HD __host__ __device__ __forceinline__
#else
#define GSIM_HD static inline
#endif

namespace gsim {

struct u32x4 { uint32_t x, y, z, w; };

GSIM_HD u32x4 philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3, uint32_t k0, uint32_t k1)
{
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        c0 = hi1 ^ c1 ^ k0;
        c1 = lo1;
        c2 = hi0 ^ c3 ^ k1;
        c3 = lo0;
        k0 += 0x9E3779B9u;
        k1 += 0xBB67AE85u;
    }
    return u32x4{c0, c1, c2, c3};
}

// Purposes (counter word 2 = topic << 8 | purpose).
enum Purpose : uint32_t {
    P_GRAFT_DLO = 1,   // getPeers for |mesh| < Dlo            gossipsub.go:1413-1427
    P_PRUNE_SHUF1 = 2, // shufflePeers before the score sort   gossipsub.go:1434
    P_PRUNE_SHUF2 = 3, // shufflePeers(plst[Dscore:])          gossipsub.go:1441
    P_GRAFT_DOUT = 4,  // getPeers for Dout top-up             gossipsub.go:1506-1512
    P_GRAFT_OPP = 5,   // getPeers for opportunistic graft     gossipsub.go:1540-1545
    P_GOSSIP = 6,      // emitGossip target shuffle            gossipsub.go:1758
    P_IWANT = 7,       // shuffleStrings(iwantlst)             gossipsub.go:687
    P_PROMISE = 8,     // rand.Intn in AddPromise              gossip_tracer.go:53
    P_GOSSIP_FILL = 9, // map order of emitGossip's Dlo fill   gossipsub.go:1739-1748
    P_GOSSIP_DUP = 10, // shuffle key of a fill duplicate      gossipsub.go:1758
    P_IHAVE_TRUNC = 11,// emitGossip's per-peer shuffleStrings  gossipsub.go:1766-1771
    P_FANOUT_NEW = 12, // Publish: getPeers for a new fanout   gossipsub.go:1020-1023 (counter word 0 = round)
    P_FANOUT = 13,     // heartbeat fanout top-up             gossipsub.go:1578-1585
    P_PX = 14,         // makePrune's getPeers (heartbeat)    gossipsub.go:1879-1882
    P_PX_GRAFT = 15,   // makePrune's getPeers (GRAFT reply)  gossipsub.go:831-834
    P_GATER = 16,      // the peer gater's rand.Float64()      peer_gater.go:357
    P_JOIN = 17,       // Join's getPeers                     gossipsub.go:1068-1092
    P_PX_LEAVE = 18,   // makePrune's getPeers (Leave's PRUNE) gossipsub.go:1118, 1866-1906
};

// Key of a choice made per (observer, other peer, message slot): the other
// peer goes into the Philox key's high word (oracle_gossip.c okey_pair).
GSIM_HD uint64_t pair_key(uint64_t seed, uint32_t tick, uint32_t observer, uint32_t topic, uint32_t purpose,
                          uint32_t slot, uint32_t other)
{
    u32x4 r = philox4x32_10(tick, observer, (topic << 8) | purpose, slot, (uint32_t)seed,
                            (uint32_t)(seed >> 32) ^ other);
    return ((uint64_t)r.x << 32) | slot;
}

// 64-bit selection key: 32 random bits above the item's row position, so keys
// are unique within a row and ties cannot occur.
GSIM_HD uint64_t select_key(uint64_t seed, uint32_t tick, uint32_t observer, uint32_t topic,
                            uint32_t purpose, uint32_t item, uint32_t pos)
{
    u32x4 r = philox4x32_10(tick, observer, (topic << 8) | purpose, item, (uint32_t)seed,
                            (uint32_t)(seed >> 32));
    return ((uint64_t)r.x << 32) | pos;
}

// PX keys (makePrune's getPeers, gossipsub.go:1879-1882): one Philox draw per
// (observer, topic, candidate) and pass, shared by every PRUNE of the topic,
// mixed (murmur3's 32-bit finaliser) with the pruned peer's row position so
// that each PRUNE's list is its own shuffle.  A hub answering hundreds of
// GRAFTs per tick draws each candidate once instead of once per PRUNE.
GSIM_HD uint32_t px_base(uint64_t seed, uint32_t tick, uint32_t observer, uint32_t topic, uint32_t purpose,
                         uint32_t item)
{
    return philox4x32_10(tick, observer, (topic << 8) | purpose, item, (uint32_t)seed, (uint32_t)(seed >> 32)).x;
}

GSIM_HD uint64_t px_key(uint32_t base, uint32_t pruned_pos, uint32_t pos)
{
    uint32_t h = base ^ ((pruned_pos + 1u) * 0x9E3779B9u);
    h ^= h >> 16;
    h *= 0x85EBCA6Bu;
    h ^= h >> 13;
    h *= 0xC2B2AE35u;
    h ^= h >> 16;
    return ((uint64_t)h << 32) | pos;
}

}  // namespace gsim
