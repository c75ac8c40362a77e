// Host interface of the GPU witness engine (csrc/witness.hip), used by the C ABI in csrc/zkfl.hip.
// Replaces circom's WASM witness calculator (tests/full_system_simulation.mjs:758-767).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <vector>

#include "field.h"

namespace zkfl {

struct WProg;  // a loaded witness program (zkfl/wprog.py image), device-resident

int wprog_load(const uint8_t* img, size_t len, hipStream_t st, WProg** out, std::string& err);
void wprog_free(WProg* p);
void wprog_info(const WProg* p, uint32_t* n_wires, uint32_t* n_inputs, uint32_t* n_public);

// input.json (circom's input format) -> flattened input signals, n_inputs x 8 u32 std form.
int wprog_inputs_json(const WProg* p, const char* json, std::vector<uint32_t>& out, std::string& err);
// same from the image bytes alone (host only, no device)
int wprog_image_inputs_json(const uint8_t* img, size_t len, const char* json, std::vector<uint32_t>& out,
                            std::string& err);

// n witnesses; inputs: n x n_inputs x 32 B std form (host); outs_host[j]: device buffer of
// n_wires std-form Fr for witness j.  ZKFL_E_CONSTRAINT when an assert fails, ZKFL_E_ARG when
// an input is not < r.
int wprog_run(const WProg* p, size_t n, const uint8_t* inputs, Fr* const* outs_host, hipStream_t st,
              std::string& err);

// Host check that every input value is < r (the ZKFL_E_ARG case of wprog_run).
bool wprog_inputs_ok(const WProg* p, size_t n, const uint8_t* inputs, std::string& err);

// Asynchronous form for pipelines (the full-prove slots): m witnesses from device inputs d_in
// (m x n_inputs x 8 u32 std) through the Montgomery scratch W (m x n_wires Fr) into d_outs[j]
// (a device array of m device pointers); d_fail[j] ends as 0xFFFFFFFF or the index of the first
// failed assert.  Nothing is synchronised; inputs must already be checked < r.
hipError_t wprog_enqueue(const WProg* p, size_t m, const uint32_t* d_in, Fr* W, Fr* const* d_outs, uint32_t* d_fail,
                         hipStream_t st);

}  // namespace zkfl
