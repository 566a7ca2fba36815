// spt_diag.h — the render kernel's diagnostic builds, selected by ONE switch (never the product
// build; `make diag` compiles all four so they stay compile-checked, and __graft_entry__.build()
// runs it):
//   -DSPT_DIAG=1  SPT_REGION_STATS: per code region, wave executions and active lanes (ballot
//                 counted), printed by spt_context_stats() to stderr
//   -DSPT_DIAG=2  SPT_WAVE_TIMES: per-wave start / end times, iterations and CU (s_memrealtime),
//                 dumped to $SPT_WAVE_DUMP; tools/wave_tail.py reads it (queue tail, residency)
//   -DSPT_DIAG=3  SPT_PROBE_SALU: SPT_PROBE_N (default 24) extra SALU per wave-iteration, the
//                 marginal issue cost of scalar work
//   -DSPT_DIAG=4  SPT_PROBE_VALU: SPT_PROBE_N extra VALU per wave-iteration (the same for vector work)
// Tuning constants with an A/B history (SPT_STEAL_MIN, SPT_GRAB, SPT_SMALL_ITERS, SPT_SMALL_UNITS,
// SPT_UNITS_PER_LANE, SPT_NUM_SGPR) are plain numbers with their measured defaults in
// spt_kernel.hip.
#pragma once
#ifndef SPT_PROBE_N
#define SPT_PROBE_N 24
#endif
#if defined(SPT_DIAG) && SPT_DIAG == 1
#define SPT_REGION_STATS 1
#elif defined(SPT_DIAG) && SPT_DIAG == 2
#define SPT_WAVE_TIMES 1
#elif defined(SPT_DIAG) && SPT_DIAG == 3
#define SPT_PROBE_SALU SPT_PROBE_N
#elif defined(SPT_DIAG) && SPT_DIAG == 4
#define SPT_PROBE_VALU SPT_PROBE_N
#elif defined(SPT_DIAG)
#error "SPT_DIAG must be 1 (region statistics), 2 (per-wave times), 3 or 4 (SALU / VALU probes)"
#endif
#if (defined(SPT_REGION_STATS) || defined(SPT_WAVE_TIMES) || defined(SPT_PROBE_SALU) || \
     defined(SPT_PROBE_VALU)) && !defined(SPT_DIAG)
#error "diagnostic builds are selected with -DSPT_DIAG=1|2|3|4 (spt_diag.h)"
#endif
