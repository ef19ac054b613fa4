// Debug-only overrides of the engine dispatch and of launch geometry: one
// table (knobs.cpp), filled once per process from RURE_AMD_DEBUG
// ("name=value,name=value", e.g. RURE_AMD_DEBUG=lex4=0,iter_chunk=4096) and
// replaced as a whole by rure_amd_debug_set (the tests and A/B tools that
// force an alternative engine).  A knob the table does not set reads -1 and
// leaves the production choice alone: no product path needs one.
#pragma once

namespace rure_amd {

enum class Knob : int {
  Lit,             // 1 / 0: the literal engine forced on / off
  Sa,              // 0: no Shift-And engine; 2: its per-lane kernel, not the tile kernel
  Lex,             // 0: no lexer engine
  Lex4,            // 0: the byte-per-step lexer table (the four-byte table's fallback)
  LexTail,         // 0: skip the lexer's tail pass (A/B of its cost; results then incomplete)
  Kmer,            // 0: the fused string-set pass on Shift-And words, not k-mer probes
  Runs,            // 0: no run engine for C+ regexes
  AsciiShadow,     // 0: no ASCII shadow automaton
  Fb,              // 0: no first-byte skip in the lexer / DFA kernels
  Prefix,          // 0: no start-state prefix skip
  Big,             // 2 / 0: the big (u32) DFA forced on / off
  BigBytes,        // the big DFA's state budget in bytes
  Lazy,            // 1 / 0: the on-demand DFA forced on / off
  LazyRows,        // rows the on-demand DFA builds ahead per round
  Lines,           // 0: no ragged line kernel
  Split,           // 0: no split is_match units
  SuffixLong,      // 0: no chunked DfaSuffix scan; 2: also below 256 KiB
  SuffixIter,      // 0: no parallel DfaSuffix find_iter; 2: also below 256 KiB
  IterLooks,       // 0: look-around regexes' find_iter on the wave path
  IterChunk,       // find_iter unit size in bytes
  IterLanes,       // find_iter lanes per CU
  IterBs,          // find_iter block size
  LongLanes,       // long-scan lanes per CU
  CoreBs,          // core-form set kernel block size
  CoreLds,         // core-form set kernel LDS budget in bytes
  CoreProf,        // 1: per-phase clock stamps of the core-form set kernel
  ScratchCap,      // bytes of cached scratch kept for reuse
  Timing,          // 1: DFA construction times on stderr
  ReplaceGeneric,  // 1: replace's generic per-block copy, not the grouped copy
  ChainSeq,        // 1: a replace_all chain step by step, not as one composed byte map
  ShadowSync,      // 1: the ASCII shadow's find_iter quit read back, not gated on the device
  IterWave,        // 0: a find_iter DFA quit sends the batch to the wave path, not to the wave-served units
  WaveCu,          // the wave-served units' waves per CU, their Pike VM lists in global scratch
  WaveSplit,       // 0: those waves' stamps in scratch too, not in the LDS
  WaveTables,      // 0: no NFA tables staged in the LDS for those waves
  WaveLds,         // 1: those waves' whole working set in the LDS, however few waves fit
  kCount
};

// The override of k, or -1.
long long knob(Knob k);

// Replaces the whole table by spec ("name=value,..."; null or "" clears it).
// Returns false (table unchanged) on an unknown name or a malformed value.
bool knob_set(const char *spec);

}  // namespace rure_amd
