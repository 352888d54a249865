// Run-time switches of the native code. Their values come from the typed, rank-checked Python
// configuration (beforeholiday_amd/config.py) through _C.set_knobs at import: no kernel or binding reads
// the environment itself, so every rank runs what its Config says (and Config.check_ranks verifies that
// all ranks agree).
#pragma once

namespace bh {

// the value set for ``name`` (dense_mfma, dense_tune, gemm_tile, gemm_log), else ``dflt``
int knob(const char* name, int dflt);
void set_knob(const char* name, int value);

}  // namespace bh
