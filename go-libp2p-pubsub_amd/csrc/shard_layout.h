// shard_layout.h — a shard's local graph and exchange bookkeeping (host side,
// not part of the ABI; see shard_plan.cpp and DESIGN.md §5).
#pragma once
#include <cstdint>
#include <string>
#include <vector>

#include "gsim.h"

namespace gsim {


struct ShardLayout {
    int32_t k = 0, K = 1;                  // this shard, shards in the job
    int64_t N = 0, E = 0;                  // global peers / edges
    std::vector<int64_t> bounds;           // [K+1] global peer range of each shard
    int64_t n_loc = 0, e_loc = 0;          // local peers / edges
    int64_t own_lo = 0, own_hi = 0;        // owned peers (local ids)
    int64_t own_e_lo = 0, own_e_hi = 0;    // local edges of the owned rows
    int64_t n_cross = 0;                   // owned-row edges into other shards
    std::vector<uint32_t> gid;             // [n_loc] global id of each local peer (ascending)
    std::vector<uint32_t> row_ptr, col;    // local CSR (symmetric)
    std::vector<uint64_t> gidx;            // [e_loc] global index of each local edge
    std::vector<int64_t> lpeer;            // [K+1] local ids of shard s's peers: [lpeer[s], lpeer[s+1])
    std::vector<int64_t> gbase, gcnt;      // [K] ghost rows of shard s's peers: local edges [gbase, gbase+gcnt)
    std::vector<std::vector<uint32_t>> crossout;   // [K] owned-row edges whose column is shard s's, edge order
    std::vector<uint32_t> xq;              // [e_loc] owned-row cross edge: its index in crossout[dest]
};

int shard_of_peer(const std::vector<int64_t>& bounds, int64_t g);
int build_layout(int64_t n, const uint32_t* row_ptr, const uint32_t* col, const int64_t* bounds, int32_t K,
                 int32_t k, ShardLayout* L, std::string* err);

}  // namespace gsim
