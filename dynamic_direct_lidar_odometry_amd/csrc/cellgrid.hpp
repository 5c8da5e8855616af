// cellgrid.hpp — build descriptor and launchers of a target's candidate cells
// (cellgrid.hip; DESIGN.md §4 "Candidate cells").
//
// A target point p is on the list of a cell C (box, expanded by `delta` for
// the lookup's fp32 cell mapping) unless
//   * its box distance to C exceeds R = min(D, bound): D = the smallest
//     farthest-corner distance of C's dominators bounds every query's nearest
//     distance, so no query of C can have p as its nearest point (or tie with
//     it); beyond the correspondence bound nothing matches anyway; or
//   * a dominator d is strictly nearer than p at every point of C: the box
//     minimum of |q - p|^2 - |q - d|^2 (linear in q) exceeds a margin that
//     covers the fp32 rounding of the search's squared distances.
// Dominators: the target points nearest to C's 8 corners and centre (any
// target points would do; nearer ones prune more).  The lists are exact
// supersets, so the lookup's (distance, position) minimum over a list equals
// the full search's, and every point at the minimum distance is on it.
#pragma once
#include <hip/hip_runtime.h>

#include "gicp_types.hpp"

namespace ddlo {

constexpr int kCgCandMax = 2048;   // candidates of one cell held in LDS (more: the cell's queries use the walk)
constexpr int kCgCounters = 16;

// counters (device, zeroed by the host before the build)
enum CgCtr {
  kCtrBand = 0,       // band cells (coarse cells within reach of the target)
  kCtrPool0 = 1,      // pool entries allocated, per level (1..4)
  kCtrSlot1 = 5,      // slots at levels 1..3 (coarse cells refined that deep)
  kCtrFinal = 8,      // final (level, slot) records
  kCtrOverflow = 9,   // coarse cells whose candidates overflowed kCgCandMax (walk)
  kCtrPoolFull = 10,  // a pool ran out (the build must be repeated with larger pools)
  kCtrFineFb = 11,    // fine cells whose list exceeds lcap (walk)
  kCtrEnt = 12,       // list entries written
  kCtrFine = 13,      // fine-table entries written
  kCtrNoMatch = 14,   // band cells without any target point within the bound
};

struct CgLevel {
  unsigned* pool;     // list members: sorted target positions
  uint2* hdr;         // per (slot, fine cell): (pool offset, count)
  int* cmax;          // per slot: the longest list of its fine cells
  int* slot_band;     // per slot: its coarse cell's band index
  int* slot_parent;   // per slot: its slot at the level above
  unsigned pool_cap;
  int slot_cap;
};

struct CgBuild {
  CloudDev tgt;
  double ox, oy, oz, s;     // grid origin and coarse cell size (the build's exact geometry)
  float fox, foy, foz, inv_s;
  int nx, ny, nz, r;        // dimensions; band radius in cells (Chebyshev)
  double delta;             // every cell box expanded by this (the lookup's fp32 cell mapping)
  double capm;              // distances beyond this (m) never match (nextafter'd bound + margin)
  double nomatch_dist;      // a non-band cell has no target point within this distance
  int lmax;                 // a level is final when all its lists have <= lmax points
  int lcap;                 // finest level: a longer list is not stored (walk)
  int* rep;                 // [ncells] a target point of each occupied cell (sorted position; INT_MAX: none)
  int* rep_tmp;             // [ncells] propagation scratch
  int* rep_final;           // [ncells] a near target point within r cells (Chebyshev), INT_MAX: none (= not band)
  unsigned long long* dir;  // [ncells] output (CellGridDev::dir)
  int* band;                // [ncells] band cell ids, 4x4x4-blocked order
  int* cnn;                 // [nband] the band cell's near target point (sorted position)
  unsigned* ctr;            // [kCgCounters]
  CgLevel lv[kCgMaxLevel + 1];
  int2* finals;             // (level, slot)
  int final_cap;
  unsigned* fin_ent;        // [finals] list entries of the final (scanned -> first entry)
  unsigned* fin_fine;       // [finals] fine cells of the final (scanned -> first fine entry)
  uint2* fine;              // output fine table
  float4* ent;              // output entries
  unsigned fine_cap, ent_cap;
};

// counters: kCgCounters lines of 32 words, then kCgShards pool counters per level
constexpr int kCgShardsHost = 16;
constexpr size_t kCgCtrWords = (size_t)(kCgCounters + (kCgMaxLevel + 1) * kCgShardsHost) * 32;

void launch_cg_occ(hipStream_t s, const CgBuild* db, int n);
void launch_cg_prop(hipStream_t s, const CgBuild* db, int axis, const int* in, int* out, long ncells);
void launch_cg_dir_fill(hipStream_t s, unsigned long long* dir, const int* band, long ncells, unsigned long long outside);
void launch_cg_band_flags(hipStream_t s, const CgBuild* db, const int* band, unsigned char* flags, long nblocked);
void launch_cg_centers(hipStream_t s, CgBuild* db, int nband);
void launch_cg_coarse(hipStream_t s, const CgBuild* db, int nband);
void launch_cg_decide(hipStream_t s, CgBuild* db, int level, int nslots, unsigned char* fl_final, unsigned char* fl_next);
void launch_cg_slots(hipStream_t s, CgBuild* db, int level, int nslots);
void launch_cg_refine(hipStream_t s, const CgBuild* db, int level, int nslots);
void launch_cg_emit_count(hipStream_t s, const CgBuild* db, int level, const int* finals, int nfinals, unsigned* ent_n,
                          unsigned* fine_n);
void launch_cg_emit_write(hipStream_t s, const CgBuild* db, int level, const int* finals, int nfinals,
                          const unsigned* ent_off, const unsigned* fine_off, unsigned ent_base, unsigned fine_base);

}  // namespace ddlo
