/*
 * zkfl.h — C ABI of the MI355X-native Groth16/BN254 prover (libzkfl.so).
 *
 * Drop-in boundary for the reference's proving path.  The reference never links a prover:
 * it shells out to snarkjs [ext].  Each entry point below replaces one
 * snarkjs operation that a host binding (N-API / ctypes) calls:
 *
 *   zkfl_zkey_load            <- snarkjs reads `<c>_final.zkey` in `groth16 prove`
 *                                (tests/full_system_simulation.mjs:773-776)
 *   zkfl_groth16_prove        <- `npx snarkjs groth16 prove <zkey> <wtns> <proof> <public>`
 *                                (tests/full_system_simulation.mjs:773-776,
 *                                 tests/quick_integration_test.mjs:426-429,
 *                                 tests/test_verified_gradient.mjs:480-483)
 *   zkfl_groth16_prove_batch  <- the sequential per-client loop
 *                                (tests/full_system_simulation.mjs:1298-1343)
 *   zkfl_setup_*              <- the bulk fixed-base work of `snarkjs groth16 setup` +
 *                                `zkey contribute` (tests/full_system_simulation.mjs:713-730)
 *   zkfl_msm_*, zkfl_ntt_*    <- ffjavascript multiExpAffine / fft as used inside
 *                                groth16 prove (exported for parity tests)
 *
 * Conventions (snarkjs/ffjavascript byte conventions):
 *   - Field elements are 32-byte little-endian.  "std" = standard form, "mont" = Montgomery
 *     form (x * 2^256 mod p), as stored in zkey sections 2-9.
 *   - Affine points: G1 = x||y (64 B), G2 = x.c0||x.c1||y.c0||y.c1 (128 B); the point at
 *     infinity is all-zero bytes.
 *   - Proof buffer (256 B): pi_a (G1) || pi_b (G2) || pi_c (G1), affine, std form — exactly
 *     the numbers snarkjs prints in proof.json (pi_a[0..1], pi_b[0..1][0..1], pi_c[0..1]).
 *   - Blinding: rs = 64 bytes (r || s, std form, < r) for deterministic parity mode, or NULL
 *     to draw r, s from the OS CSPRNG (snarkjs draws them with Fr.random()).
 * All functions return 0 on success and a negative ZKFL_E_* code on failure; the message is
 * in zkfl_last_error() (thread-local).  A context is bound to one device and one stream;
 * contexts are independent (multi-GPU = one context per device, one process per GPU).
 */
#ifndef ZKFL_H
#define ZKFL_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZKFL_OK 0
#define ZKFL_E_ARG -1        /* bad argument / null pointer */
#define ZKFL_E_FORMAT -2     /* malformed zkey / wtns / r1cs bytes */
#define ZKFL_E_PRIME -3      /* file prime is not BN254 r / q */
#define ZKFL_E_MISMATCH -4   /* nWitness != nVars, wrong section sizes */
#define ZKFL_E_DEVICE -5     /* HIP runtime error / no GPU */
#define ZKFL_E_OOM -6        /* device allocation failed */
#define ZKFL_E_CONSTRAINT -7 /* witness does not satisfy the circuit */

typedef struct zkfl_ctx zkfl_ctx;
typedef struct zkfl_key zkfl_key;
typedef struct zkfl_witness zkfl_witness;
typedef struct zkfl_wprog zkfl_wprog;

int zkfl_version(void);
/* First 16 hex digits of SHA-256 over the sources this library was built from (the csrc .h, .hip
 * and .cc files sorted by name, then include/zkfl.h; the package Makefile).  bench.py prints it and smoke()
 * checks it against the tree it runs from (zkfl/native.py::source_id). */
const char* zkfl_build_id(void);
const char* zkfl_last_error(void);
int zkfl_device_count(int* count);

int zkfl_ctx_create(int device, zkfl_ctx** out);
int zkfl_ctx_destroy(zkfl_ctx* ctx);
/* Per-kernel timing with HIP events on the stream each kernel runs on (bench.py roofline).
 * enabled: 0 off, 1 on, 2 on + serialized (a proof's G2 and assembly work is put on its main
 * stream, so with one slot every kernel runs alone and its events time it in isolation). */
int zkfl_ctx_set_profiling(zkfl_ctx* ctx, int enabled);
/* name: "msm_accumulate_g1", "msm_accumulate_g2", "ntt", "abc", "prove", "witness" (full-prove
 * slots).  Synchronises the device.
 * total_ms: summed event time; units: summed algorithmic units (MSM entries, NTT elements...);
 * median_ms (nullable): median single-launch time, robust to a one-off stalled dispatch. */
int zkfl_ctx_profile(zkfl_ctx* ctx, const char* name, double* total_ms, uint64_t* launches, double* units,
                     double* median_ms);
int zkfl_ctx_profile_reset(zkfl_ctx* ctx);
int zkfl_ctx_synchronize(zkfl_ctx* ctx);

/* Parse a snarkjs groth16 .zkey and make it device-resident (bases expanded per window).
 * The caller keeps ownership of buf. */
int zkfl_zkey_load(zkfl_ctx* ctx, const uint8_t* buf, size_t len, zkfl_key** out);
/* The same key by path, in two steps so a host can overlap them with creating its context:
 * zkfl_zkey_file_open maps the file (read-only) and parses it on host threads -- no device work --,
 * zkfl_zkey_load_file makes it device-resident (= zkfl_zkey_load on the file's bytes),
 * zkfl_zkey_file_close unmaps it (any time after the load).  snarkjs reads the key by file name:
 * `snarkjs groth16 prove <zkey> ...` (tests/full_system_simulation.mjs:773-776); node/snarkjs_shim.js
 * maps it while its HIP context comes up.  Errors: ZKFL_E_ARG (open / map failed), as zkfl_zkey_load. */
typedef struct zkfl_zkey_file zkfl_zkey_file;
int zkfl_zkey_file_open(const char* path, zkfl_zkey_file** out);
int zkfl_zkey_load_file(zkfl_ctx* ctx, const zkfl_zkey_file* f, zkfl_key** out);
int zkfl_zkey_file_close(zkfl_zkey_file* f);
int zkfl_key_free(zkfl_key* key);
int zkfl_key_info(const zkfl_key* key, uint32_t* n_vars, uint32_t* n_public, uint32_t* domain_size);
/* Number of proofs kept in flight by zkfl_groth16_prove_batch (1..32, default 3).  Each slot
 * owns one HIP stream and its own scratch (~0.6 GB for the 2^18 training circuit); proofs in
 * different slots overlap on the GPU.  HIP maps a process's streams onto GPU_MAX_HW_QUEUES
 * hardware queues (HIP default 4, which the GPU boxes export): set it in the environment before
 * the first HIP call to at least the slot count, or the slots serialize.  Measured on MI355X
 * (bench.py's default): 20 slots over 28 queues is the best configuration; 24+
 * slots or 32 queues oversubscribe the hardware queues and lose throughput. */
int zkfl_key_set_slots(zkfl_key* key, int slots);

/* Full prove from a .wtns byte image (host).  pub_out may be NULL; otherwise receives
 * n_public x 32 B std-form public signals (witness[1..n_public]) and *npub their count. */
int zkfl_groth16_prove(zkfl_ctx* ctx, zkfl_key* key, const uint8_t* wtns, size_t wtns_len,
                       const uint8_t* rs, uint8_t proof_out[256], uint8_t* pub_out, size_t* npub);

/* Device-resident witnesses (steady-state proving: input already in HBM). */
int zkfl_witness_upload(zkfl_ctx* ctx, const zkfl_key* key, const uint8_t* wtns, size_t wtns_len,
                        zkfl_witness** out);
int zkfl_witness_free(zkfl_witness* w);
int zkfl_groth16_prove_resident(zkfl_ctx* ctx, zkfl_key* key, const zkfl_witness* w, const uint8_t* rs,
                                uint8_t proof_out[256]);
/* n independent proofs (rs: n x 64 B or NULL); proofs_out: n x 256 B. */
int zkfl_groth16_prove_batch(zkfl_ctx* ctx, zkfl_key* key, size_t n, const zkfl_witness* const* w,
                             const uint8_t* rs, uint8_t* proofs_out);

/* Multi-key batch: proof i uses keys[i] and witness w[i] (uploaded for keys[i]); rs: n x 64 B or
 * NULL; proofs_out: n x 256 B.  Replaces the reference's per-round loop that proves each client's
 * training update and then its secure-aggregation update with two different zkeys
 * (tests/full_system_simulation.mjs:1298-1343: `trainAndGenerateProof` -> groth16 prove of
 * sgd_verified_final.zkey, :773-776; `generateSecureAggregationProof` -> groth16 prove of the
 * secure_masked_update zkey, :1040-1107).  Every key keeps its own proof slots resident; the jobs
 * are issued in order, each on the next slot of its key, so proofs of different circuits
 * overlap on the device. */
int zkfl_groth16_prove_multi(zkfl_ctx* ctx, size_t n, zkfl_key* const* keys, const zkfl_witness* const* w,
                             const uint8_t* rs, uint8_t* proofs_out);

/* One proof split across GPUs (optional row: a proof too large for one device's
 * latency budget).  The reference proves each client on one CPU (`groth16 prove`,
 * tests/full_system_simulation.mjs:773-776); these calls divide that same prove over G processes,
 * one per GPU, with the caller's all-gather in between (zkfl/split.py: torch.distributed; RCCL or gloo):
 *
 *   zkfl_zkey_load_shard   every rank loads the same zkey keeping base i of each query (A, B1, B2,
 *                          C, H) only when i % n_shards == shard, and the alpha/beta/delta
 *                          augmentation bases only on shard 0.  The QAP rows and NTT are whole.
 *   zkfl_groth16_prove_part_batch   per rank, per proof: ABC + coset NTT over the FULL witness
 *                          (h is needed whole; redundant on every rank, ~0.4 ms), then this shard's
 *                          share of the five MSMs.  rs is REQUIRED (n x 64 B, the same r, s on every
 *                          rank: rank 0 draws them and broadcasts).  parts_out: n x 768 B =
 *                          A' (128) | B1' (128) | B2' (256) | C' (128) | H (128), each an XYZZ point
 *                          (x = X/ZZ, y = Y/ZZZ; G1: X|Y|ZZ|ZZZ, G2: the same with c0|c1 per
 *                          coordinate), every coordinate 32 B std-form LE, ZZ = 0 is infinity --
 *                          projective, so a shard pays no inversion; the alpha/beta/delta/r/s terms
 *                          are on shard 0; C' may already include H, then H = infinity.
 *   zkfl_groth16_assemble  after the all_gather: parts = n x n_parts x 768 B (proof-major); the parts
 *                          of each proof are summed and pi_c = C' + H + s pi_a + r B1' is formed on
 *                          the GPU -> n x 256 B proofs, byte-identical to zkfl_groth16_prove_batch
 *                          with the same r, s.  Needs no key.  A coordinate >= q -> ZKFL_E_ARG. */
int zkfl_zkey_load_shard(zkfl_ctx* ctx, const uint8_t* buf, size_t len, uint32_t shard, uint32_t n_shards,
                         zkfl_key** out);
int zkfl_key_shard(const zkfl_key* key, uint32_t* shard, uint32_t* n_shards);
int zkfl_groth16_prove_part_batch(zkfl_ctx* ctx, zkfl_key* key, size_t n, const zkfl_witness* const* w,
                                  const uint8_t* rs, uint8_t* parts_out);
int zkfl_groth16_assemble(zkfl_ctx* ctx, size_t n, size_t n_parts, const uint8_t* parts, const uint8_t* rs,
                          uint8_t* proofs_out);

/* Parity hooks: the deterministic core of one proof.
 * h_out: domain_size x 32 B std (coset evaluations a*b-c, the H-MSM scalars) or NULL;
 * msm_out: A (64) | B1 (64) | B2 (128) | C (64) | H (64) std affine MSM results over the
 * zkey queries *without* the alpha/beta/delta/r/s terms, or NULL. */
int zkfl_debug_prove_parts(zkfl_ctx* ctx, zkfl_key* key, const uint8_t* wtns, size_t wtns_len, uint8_t* h_out,
                           uint8_t* msm_out);

/* GLV split used by the proof assembly (host code, no device): k (32 B std, < r) ->
 * out = k1 || k2, each 20 B: |k_i| (16 B little-endian) then a u32 sign (1 = negative), with
 * k = k1 + k2 * lambda (mod r), |k_i| < 2^128 (csrc/glv.h; tests/test_abi.py checks it). */
int zkfl_debug_glv_split(const uint8_t k[32], uint8_t out[40]);

/* The assembly's scalar multiplication on the device (parity hook): out[i] = k_i * P_i for n pairs,
 * P_i affine std (64 B, (0, 0) = infinity), k_i 32 B std < r, out affine std (infinity = zeros) --
 * the GLV halves of k_i as two row-distributed chains, summed, affine by the divsteps inverse, as
 * k_assemble computes s pi_A + r B1 (no reference counterpart: snarkjs's G1.timesFr inside
 * groth16_prove). */
int zkfl_debug_g1_glv_mul(zkfl_ctx* ctx, size_t n, const uint8_t* points, const uint8_t* scalars, uint8_t* out);

/* Wave-level kernel timeline (measurement only; libraries built with -DZK_WTRACE=1, otherwise every
 * op returns ZKFL_E_ARG).  op 1: start recording into a fresh device buffer of `cap` records (any
 * earlier one is freed); op 2: wait for the device, stop recording, copy min(count, cap) records of
 * 40 B {u32 kind, u32 HW_ID, u64 start, u64 end (s_memrealtime, 100 MHz), u64 start, u64 end
 * (s_memtime, shader clock cycles)} to out (may be NULL) and the number recorded (possibly > cap) to
 * *count; op 0: free.  tools/wtrace.py reads them. */
int zkfl_debug_wtrace(zkfl_ctx* ctx, int op, uint32_t cap, void* out, uint32_t* count);

/* Stand-alone primitives (parity tests).  bases: mont affine; scalars: std, n x 32 B. */
int zkfl_msm_g1(zkfl_ctx* ctx, const uint8_t* bases, const uint8_t* scalars, size_t n, uint8_t out[64]);
int zkfl_msm_g2(zkfl_ctx* ctx, const uint8_t* bases, const uint8_t* scalars, size_t n, uint8_t out[128]);
/* In place: 2^logn std-form evaluations on the domain -> evaluations on the odd coset
 * (snarkjs ifft + batchApplyKey(inc) + fft). */
int zkfl_ntt_coset(zkfl_ctx* ctx, uint8_t* data, uint32_t logn);

/* Witness generation on the GPU (replaces circom's WASM witness calculator:
 * `node <c>_js/generate_witness.cjs <c>.wasm input.json out.wtns`, tests/full_system_simulation.mjs:758-767,
 * and `snarkjs wtns calculate`, tests/test_secureagg.cjs:108-118).  The circuit is a witness
 * program image compiled once per circuit by zkfl/wprog.py (the .wasm's role); inputs are the
 * circuit's input signals in declaration order, flattened, reduced mod r, 32 B std form each
 * (zkfl/wprog.py::input_bytes does the input.json -> bytes step).  An unsatisfied assert returns
 * ZKFL_E_CONSTRAINT (circom: "Assert Failed"); an input >= r returns ZKFL_E_ARG. */
int zkfl_wprog_load(zkfl_ctx* ctx, const uint8_t* prog, size_t len, zkfl_wprog** out);
int zkfl_wprog_free(zkfl_wprog* prog);
int zkfl_wprog_info(const zkfl_wprog* prog, uint32_t* n_wires, uint32_t* n_inputs, uint32_t* n_public);
/* Byte size of one .wtns image for this program (snarkjs wtns v2: 76 + 32 x n_wires). */
size_t zkfl_wtns_size(const zkfl_wprog* prog);
/* circom's input.json (one object of signal name -> number | decimal/0x string | nested arrays;
 * negatives reduced mod r) -> the flattened input vector, using the signal table of a program
 * image.  Host only (no device needed).  inputs_out: room for `cap` values of 32 B; *n_inputs
 * receives the count.  Missing signal / wrong shape / non-integer -> ZKFL_E_ARG. */
int zkfl_wprog_parse_inputs(const uint8_t* prog, size_t len, const char* input_json, uint8_t* inputs_out, size_t cap,
                            size_t* n_inputs);
/* One witness from input.json -> one .wtns image (the generate_witness.cjs call, :758-767). */
int zkfl_witness_compute_json(zkfl_ctx* ctx, const zkfl_wprog* prog, const char* input_json, uint8_t* wtns_out);
/* n witnesses -> n .wtns images at wtns_out + i * zkfl_wtns_size(prog). */
int zkfl_witness_compute(zkfl_ctx* ctx, const zkfl_wprog* prog, size_t n, const uint8_t* inputs, uint8_t* wtns_out);
/* n witnesses computed straight into device-resident witnesses for `key` (no host round trip). */
int zkfl_witness_compute_resident(zkfl_ctx* ctx, const zkfl_wprog* prog, const zkfl_key* key, size_t n,
                                  const uint8_t* inputs, zkfl_witness** out);

/* Full prove, pipelined (snarkjs `groth16.fullProve(input, wasm, zkey)` for a batch; the
 * reference's per-client loop `generate_witness.cjs` + `groth16 prove`,
 * tests/full_system_simulation.mjs:758-776 and :1298-1343).  The witnesses are computed a group
 * of `slots` clients at a time (one batched run of the witness engine on the key's witness
 * stream, straight into HBM), one group ahead of the proof slots that consume them, so witness
 * generation overlaps the MSMs of the previous group; nothing returns to the host but the proofs
 * and the public signals.  inputs: n x n_inputs x 32 B std (zkfl_wprog_parse_inputs per input.json);
 * rs: n x 64 B or NULL (CSPRNG); proofs_out: n x 256 B; pubs_out: n x nPublic x 32 B or NULL.
 * A witness whose asserts fail gives ZKFL_E_CONSTRAINT naming the first such index (its proof
 * bytes are zeroed, the others are valid); an input >= r gives ZKFL_E_ARG before any work. */
int zkfl_groth16_full_prove_batch(zkfl_ctx* ctx, zkfl_key* key, const zkfl_wprog* prog, size_t n,
                                  const uint8_t* inputs, const uint8_t* rs, uint8_t* proofs_out, uint8_t* pubs_out);

/* snarkjs `groth16.fullProve(input, wasm, zkey)` for one input.json text: parsed against the loaded
 * program's signal table, then the full-prove pipeline above with n = 1.  pub_out: nPublic x 32 B
 * or NULL.  Errors as zkfl_wprog_parse_inputs (ZKFL_E_ARG) and zkfl_groth16_full_prove_batch. */
int zkfl_groth16_full_prove_json(zkfl_ctx* ctx, zkfl_key* key, const zkfl_wprog* prog, const char* input_json,
                                 const uint8_t* rs, uint8_t proof_out[256], uint8_t* pub_out);

/* snarkjs `groth16.fullProve` over n input.json texts (the reference runs one fullProve /
 * `generate_witness.cjs` + `groth16 prove` pair per client, tests/full_system_simulation.mjs:758-776):
 * host worker threads parse the texts against the program's signal table ahead of the slot
 * scheduler (at most 64 parsed vectors held), so parsing overlaps the proofs in flight; then the
 * zkfl_groth16_full_prove_batch pipeline.  Errors: a text that does not parse or does not fill
 * the program's inputs gives ZKFL_E_ARG naming its index (proofs of earlier slot groups complete);
 * otherwise as zkfl_groth16_full_prove_batch. */
int zkfl_groth16_full_prove_json_batch(zkfl_ctx* ctx, zkfl_key* key, const zkfl_wprog* prog, size_t n,
                                       const char* const* input_jsons, const uint8_t* rs, uint8_t* proofs_out,
                                       uint8_t* pubs_out);

/* Multi-key full prove: job i = (keys[i], progs[i], inputs[i] = that program's input vector);
 * pubs_out[i] (or pubs_out NULL) receives keys[i]'s nPublic x 32 B.  Same error behaviour as
 * zkfl_groth16_full_prove_batch; the witness index in a ZKFL_E_CONSTRAINT message is the job index. */
int zkfl_groth16_full_prove_multi(zkfl_ctx* ctx, size_t n, zkfl_key* const* keys, const zkfl_wprog* const* progs,
                                  const uint8_t* const* inputs, const uint8_t* rs, uint8_t* proofs_out,
                                  uint8_t* const* pubs_out);

/* Verification (replaces `snarkjs groth16 verify <vkey> <public> <proof>`,
 * tests/full_system_simulation.mjs:865-868; snarkjs groth16_verify, restated in
 * oracle/groth16.py::verify).  vk image (see zkfl/groth16.py::vk_bytes for vkey.json -> bytes):
 *   nPublic u32 LE | alpha1 (64) | beta2 (128) | gamma2 (128) | delta2 (128) | IC[nPublic+1] (64 each),
 * standard-form affine LE, G2 as x.c0|x.c1|y.c0|y.c1 (the proof's encoding).  pub: npub x 32 B std.
 * Returns 1 (valid), 0 (invalid: pairing check fails, a public signal >= r, a proof coordinate
 * >= q, a point off its curve, pi_b outside the order-r subgroup) or a negative ZKFL_E_* code
 * (malformed vk, npub != nPublic).  The prepared key is cached in the context. */
int zkfl_groth16_verify(zkfl_ctx* ctx, const uint8_t* vk, size_t vk_len, const uint8_t* pub, size_t npub,
                        const uint8_t proof[256]);
/* n proofs against one key, one GPU lane each: pubs n x npub x 32 B, proofs n x 256 B,
 * results[i] = 1 / 0.  Returns ZKFL_OK or an error code. */
int zkfl_groth16_verify_batch(zkfl_ctx* ctx, const uint8_t* vk, size_t vk_len, size_t n, const uint8_t* pubs,
                              size_t npub, const uint8_t* proofs, int32_t* results);
/* Optimal-ate pairing e(P_i, Q_i) for n pairs (g1: n x 64 B, g2: n x 128 B, std affine; all-zero
 * = infinity).  gt_out: n x 384 B, 12 std-form Fq in the ffjavascript Fq12 toObject order
 * (c0.c0.a, c0.c0.b, c0.c1.a, ... c1.c2.b) -- the layout of vkey.json's vk_alphabeta_12. */
int zkfl_pairing(zkfl_ctx* ctx, size_t n, const uint8_t* g1, const uint8_t* g2, uint8_t* gt_out);
/* Parity hook: the Miller-loop value before the final exponentiation, same layout. */
int zkfl_debug_miller_loop(zkfl_ctx* ctx, size_t n, const uint8_t* g1, const uint8_t* g2, uint8_t* out);

/* Poseidon hashing and Merkle trees on the GPU: the reference's data/server side
 * (tests/full_system_simulation.mjs:139-238, circomlibjs `poseidon` [ext]), bit-identical to
 * circomlib Poseidon (src/circuits/lib/poseidon.circom:35-96).  Values are 32 B std-form LE, < r
 * (ZKFL_E_ARG otherwise); circomlibjs reduces wider integers mod r, callers do that first.
 *
 * zkfl_poseidon_params (host only, no device): circomlib's constants for width t = 2..17 as the
 * Grain LFSR generates them -- (8 + R_P) * t raw round constants and the 2t Cauchy points x|y of the
 * MDS M[i][j] = 1/(x_i + y_j), std form -- and R_P.  Either output may be NULL. */
int zkfl_poseidon_params(uint32_t t, uint8_t* consts_out, uint8_t* xy_out, uint32_t* rp_out);
/* out[i] = Poseidon(inputs[i*arity .. +arity)), arity 1..16 (circomlibjs poseidon(inputs)). */
int zkfl_poseidon_batch(zkfl_ctx* ctx, uint32_t arity, size_t n, const uint8_t* inputs, uint8_t* out);
/* out[i] = vectorHash(values[i*len .. +len)), len 1..256: Poseidon of <= 16 values, else Poseidon of
 * the 16-value chunk hashes (vectorHash, tests/full_system_simulation.mjs:139-156; VectorHash,
 * src/circuits/training/vector_hash.circom:46-89). */
int zkfl_vector_hash_batch(zkfl_ctx* ctx, uint32_t len, size_t n, const uint8_t* values, uint8_t* out);
/* buildMerkleTree(leafHashes, depth) (tests/full_system_simulation.mjs:198-223): n <= 2^depth leaves
 * padded with Poseidon([0]), depth <= ZKFL_MERKLE_MAX_DEPTH.  tree_out: (2^(depth+1) - 1) x 32 B, the
 * reference's `tree` array flattened -- level 0 (2^depth padded leaves) first, the root last, so
 * getMerkleProof (:225-238) reads tree_out[level_offset(l) + (idx >> l ^ 1)]. */
#define ZKFL_MERKLE_MAX_DEPTH 30
int zkfl_merkle_build(zkfl_ctx* ctx, const uint8_t* leaves, size_t n, uint32_t depth, uint8_t* tree_out);
/* computeDatasetCommitment (tests/full_system_simulation.mjs:309-335) without leaving the device:
 * leaf i = vectorHash(values[i*len .. +len)) (features[i] || label[i]), then buildMerkleTree;
 * root_D = the last 32 B of tree_out. */
int zkfl_dataset_commit(zkfl_ctx* ctx, const uint8_t* values, size_t n, uint32_t len, uint32_t depth,
                        uint8_t* tree_out);

/* Dev-ceremony fixed-base multiplications: out[i] = scalars[i] * generator, mont affine. */
int zkfl_setup_g1_gen_mul(zkfl_ctx* ctx, const uint8_t* scalars, size_t n, uint8_t* out);
int zkfl_setup_g2_gen_mul(zkfl_ctx* ctx, const uint8_t* scalars, size_t n, uint8_t* out);

/* Ceremony primitives: the bulk group work of the snarkjs setup commands the reference runs once
 * per circuit (tests/test_secureagg.cjs:25-57: `powersoftau new|contribute|prepare phase2`,
 * `groth16 setup`; tests/full_system_simulation.mjs:713-730: `groth16 setup`, `zkey contribute`).
 * The file handling around them is zkfl/ptau.py.  Points are mont affine
 * (the LEM bytes of ptau / zkey sections; infinity = all zero), scalars std 32 B LE; G2 points are
 * x.c0|x.c1|y.c0|y.c1 (128 B).
 *
 * out[i] = scalars[i] * points[i]: `powersoftau contribute` (tauG1[i] *= tau^i, ...) and
 * `zkey contribute` (delta *= d, C and H *= 1/d). */
int zkfl_setup_g1_scale(zkfl_ctx* ctx, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out);
int zkfl_setup_g2_scale(zkfl_ctx* ctx, const uint8_t* points, const uint8_t* scalars, size_t n, uint8_t* out);
/* out[j] = (1/N) sum_i w^-ij points[i], N = 2^logn (logn <= 28), w = Fr.w[logn] (ffjavascript:
 * nqr = 5): the inverse FFT over the group that `powersoftau prepare phase2` applies to each
 * 2^p prefix of tauG1 / tauG2 / alphaTauG1 / betaTauG1 (ptau sections 12-15), i.e. L_j(tau) G. */
int zkfl_setup_g1_lagrange(zkfl_ctx* ctx, const uint8_t* points, uint32_t logn, uint8_t* out);
int zkfl_setup_g2_lagrange(zkfl_ctx* ctx, const uint8_t* points, uint32_t logn, uint8_t* out);
/* Sparse combinations out[r] = sum_{t in [rowptr[r], rowptr[r+1])} coefs[t] * bases[idx[t]]
 * (rowptr: n_out + 1 entries, rowptr[0] = 0, < 2^32 - 1 terms; idx[t] < n_bases; empty row ->
 * infinity): `groth16 setup`'s A_i, B1_i, B2_i, C_i, IC_i from the Lagrange bases. */
int zkfl_setup_g1_lincomb(zkfl_ctx* ctx, const uint8_t* bases, size_t n_bases, size_t n_out, const uint64_t* rowptr,
                          const uint32_t* idx, const uint8_t* coefs, uint8_t* out);
int zkfl_setup_g2_lincomb(zkfl_ctx* ctx, const uint8_t* bases, size_t n_bases, size_t n_out, const uint64_t* rowptr,
                          const uint32_t* idx, const uint8_t* coefs, uint8_t* out);

#ifdef __cplusplus
}
#endif
#endif /* ZKFL_H */
