// Per-phase single-pass chain kernels, unit 2 of 4 (chain_pp.h, chain_pp_unit.inc).
#define PP_UNIT 2
#include "chain_pp_unit.inc"
