// N-API binding of libzkfl (include/zkfl.h) for a Node.js host.
//
// Replaces the child-process boundary of the reference harness
// (`execSync("npx snarkjs groth16 prove ...")`, tests/full_system_simulation.mjs:773-776):
// a Node process loads the proving key once and proves in-process.  Proving runs on a libuv
// worker thread (napi_create_async_work) so the event loop is not blocked, and resolves a
// Promise like snarkjs's `groth16.prove`.
//
// JS surface (see snarkjs_shim.js):
//   version() -> number
//   deviceCount() -> number
//   createContext(device) -> ctx      (created on a thread of its own: the call returns at once and
//                                      the first use waits for it, so a CLI maps its key meanwhile)
//   loadKey(ctx, zkeyBuffer) -> key                       (zkfl_zkey_load)
//   openKeyFile(path) -> file                             (zkfl_zkey_file_open: map + host parse)
//   loadKeyFile(ctx, file) -> key                         (zkfl_zkey_load_file)
//   contextReady(ctx) -> true                             (waits for the context; throws if it failed)
//   quickExit(code)                                       (the CLI's exit: _exit after stdio flush)
//   keyInfo(key) -> {nVars, nPublic, domainSize}
//   prove(ctx, key, wtnsBuffer[, rsBuffer]) -> Promise<{proof: Buffer(256), publicSignals: Buffer}>
//   verify(ctx, vkBuffer, publicBuffer, proofBuffer) -> Promise<boolean>   (zkfl_groth16_verify)
//   loadProgram(ctx, zkwpBuffer) -> prog                                   (zkfl_wprog_load)
//   witness(ctx, prog, inputJsonString) -> Promise<Buffer(.wtns)>          (zkfl_witness_compute_json)
//   fullProve(ctx, key, prog, inputJsonString[, rsBuffer])
//       -> Promise<{proof: Buffer(256), publicSignals: Buffer}>           (zkfl_groth16_full_prove_json)
//   pairing(ctx, g1Buffer(64), g2Buffer(128)) -> Buffer(384)              (zkfl_pairing, vk_alphabeta_12)
//   poseidon / vectorHash / merkleBuild                                    (node/circomlibjs, see below)
#include <node_api.h>

#include <unistd.h>

#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "zkfl.h"

namespace {

napi_value throw_err(napi_env env, int rc) {
  std::string msg = std::string("zkfl error ") + std::to_string(rc) + ": " + zkfl_last_error();
  napi_throw_error(env, nullptr, msg.c_str());
  return nullptr;
}

napi_value Version(napi_env env, napi_callback_info) {
  napi_value v;
  napi_create_int32(env, zkfl_version(), &v);
  return v;
}

napi_value DeviceCount(napi_env env, napi_callback_info) {
  int c = 0;
  zkfl_device_count(&c);
  napi_value v;
  napi_create_int32(env, c, &v);
  return v;
}

// A context being created on its own thread (hipInit and the device's context take ~80 ms of a
// CLI run); get() waits for it.
struct CtxBox {
  std::thread th;
  zkfl_ctx* ctx = nullptr;
  int rc = 0;
  std::string err;
  zkfl_ctx* get() {
    if (th.joinable()) th.join();
    return ctx;
  }
};

// argv value -> the context (waiting for its creation); throws and returns nullptr when it failed.
// Every entry point that takes a context goes through here, so a failed creation (no device, out
// of memory) surfaces with its own code and message rather than as a null-context error.
zkfl_ctx* ctx_arg(napi_env env, napi_value v) {
  void* data = nullptr;
  if (napi_get_value_external(env, v, &data) != napi_ok || !data) return nullptr;
  CtxBox* b = static_cast<CtxBox*>(data);
  zkfl_ctx* c = b->get();
  if (!c) {
    std::string msg = std::string("zkfl error ") + std::to_string(b->rc) + ": " + b->err;
    napi_throw_error(env, nullptr, msg.c_str());
  }
  return c;
}

// Finalizers run in an unspecified order; the C ABI keeps the context alive while keys and
// programs made on it live (zkfl_ctx_destroy drops only the handle's reference), so any order is safe.
void ctx_finalize(napi_env, void* data, void*) {
  CtxBox* b = static_cast<CtxBox*>(data);
  zkfl_ctx_destroy(b->get());
  delete b;
}
void file_finalize(napi_env, void* data, void*) { zkfl_zkey_file_close(static_cast<zkfl_zkey_file*>(data)); }
void key_finalize(napi_env, void* data, void*) { zkfl_key_free(static_cast<zkfl_key*>(data)); }
void prog_finalize(napi_env, void* data, void*) { zkfl_wprog_free(static_cast<zkfl_wprog*>(data)); }

napi_value CreateContext(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  int32_t dev = 0;
  if (argc >= 1) napi_get_value_int32(env, argv[0], &dev);
  CtxBox* b = new CtxBox();
  b->th = std::thread([b, dev] {
    b->rc = zkfl_ctx_create(dev, &b->ctx);
    if (b->rc) b->err = zkfl_last_error();
  });
  napi_value ext;
  napi_create_external(env, b, ctx_finalize, nullptr, &ext);
  return ext;
}

napi_value LoadKey(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  void* ctx = nullptr;
  void* data = nullptr;
  size_t len = 0;
  if (argc < 2 || napi_get_value_external(env, argv[0], &ctx) != napi_ok ||
      napi_get_buffer_info(env, argv[1], &data, &len) != napi_ok) {
    napi_throw_type_error(env, nullptr, "loadKey(ctx, zkeyBuffer)");
    return nullptr;
  }
  zkfl_ctx* c = ctx_arg(env, argv[0]);
  if (!c) return nullptr;
  zkfl_key* key = nullptr;
  int rc = zkfl_zkey_load(c, static_cast<const uint8_t*>(data), len, &key);
  if (rc) return throw_err(env, rc);
  napi_value ext;
  napi_create_external(env, key, key_finalize, nullptr, &ext);
  return ext;
}

napi_value OpenKeyFile(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  size_t n = 0;
  if (argc < 1 || napi_get_value_string_utf8(env, argv[0], nullptr, 0, &n) != napi_ok) {
    napi_throw_type_error(env, nullptr, "openKeyFile(path)");
    return nullptr;
  }
  std::string path(n, '\0');
  napi_get_value_string_utf8(env, argv[0], &path[0], n + 1, &n);
  zkfl_zkey_file* f = nullptr;
  int rc = zkfl_zkey_file_open(path.c_str(), &f);
  if (rc) return throw_err(env, rc);
  napi_value ext;
  napi_create_external(env, f, file_finalize, nullptr, &ext);
  return ext;
}

napi_value LoadKeyFile(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  void* f = nullptr;
  if (argc < 2 || napi_get_value_external(env, argv[1], &f) != napi_ok) {
    napi_throw_type_error(env, nullptr, "loadKeyFile(ctx, file)");
    return nullptr;
  }
  zkfl_ctx* c = ctx_arg(env, argv[0]);
  if (!c) return nullptr;
  zkfl_key* key = nullptr;
  int rc = zkfl_zkey_load_file(c, static_cast<const zkfl_zkey_file*>(f), &key);
  if (rc) return throw_err(env, rc);
  napi_value ext;
  napi_create_external(env, key, key_finalize, nullptr, &ext);
  return ext;
}

napi_value ContextReady(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  if (argc < 1 || !ctx_arg(env, argv[0])) return nullptr;
  napi_value t;
  napi_get_boolean(env, true, &t);
  return t;
}

// quickExit(code): stdio flushed, then _exit (no atexit handlers, no static destructors)
napi_value QuickExit(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  int32_t code = 0;
  if (argc >= 1) napi_get_value_int32(env, argv[0], &code);
  fflush(nullptr);
  _exit(code);
}

napi_value KeyInfo(napi_env env, napi_callback_info info) {
  size_t argc = 1;
  napi_value argv[1];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  void* key = nullptr;
  if (argc < 1 || napi_get_value_external(env, argv[0], &key) != napi_ok) {
    napi_throw_type_error(env, nullptr, "keyInfo(key)");
    return nullptr;
  }
  uint32_t nv = 0, np = 0, dom = 0;
  int rc = zkfl_key_info(static_cast<zkfl_key*>(key), &nv, &np, &dom);
  if (rc) return throw_err(env, rc);
  napi_value obj, a, b, c;
  napi_create_object(env, &obj);
  napi_create_uint32(env, nv, &a);
  napi_create_uint32(env, np, &b);
  napi_create_uint32(env, dom, &c);
  napi_set_named_property(env, obj, "nVars", a);
  napi_set_named_property(env, obj, "nPublic", b);
  napi_set_named_property(env, obj, "domainSize", c);
  return obj;
}

struct ProveWork {
  napi_async_work work = nullptr;
  napi_deferred deferred = nullptr;
  zkfl_ctx* ctx = nullptr;
  zkfl_key* key = nullptr;
  std::vector<uint8_t> wtns, rs;
  uint8_t proof[256];
  std::vector<uint8_t> pub;
  size_t npub = 0;
  int rc = 0;
  std::string err;
};

void prove_execute(napi_env, void* data) {
  ProveWork* w = static_cast<ProveWork*>(data);
  uint32_t nv = 0, np = 0, dom = 0;
  zkfl_key_info(w->key, &nv, &np, &dom);
  w->pub.resize((size_t)np * 32 + 32);
  w->rc = zkfl_groth16_prove(w->ctx, w->key, w->wtns.data(), w->wtns.size(), w->rs.empty() ? nullptr : w->rs.data(),
                             w->proof, w->pub.data(), &w->npub);
  if (w->rc) w->err = zkfl_last_error();
}

void prove_complete(napi_env env, napi_status, void* data) {
  ProveWork* w = static_cast<ProveWork*>(data);
  if (w->rc) {
    napi_value msg, err;
    std::string m = "zkfl prove failed (" + std::to_string(w->rc) + "): " + w->err;
    napi_create_string_utf8(env, m.c_str(), NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, nullptr, msg, &err);
    napi_reject_deferred(env, w->deferred, err);
  } else {
    napi_value obj, proof, pub;
    void* p;
    napi_create_buffer_copy(env, 256, w->proof, &p, &proof);
    napi_create_buffer_copy(env, w->npub * 32, w->pub.data(), &p, &pub);
    napi_create_object(env, &obj);
    napi_set_named_property(env, obj, "proof", proof);
    napi_set_named_property(env, obj, "publicSignals", pub);
    napi_resolve_deferred(env, w->deferred, obj);
  }
  napi_delete_async_work(env, w->work);
  delete w;
}

napi_value Prove(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  void *ctx = nullptr, *key = nullptr, *wt = nullptr, *rs = nullptr;
  size_t wlen = 0, rslen = 0;
  if (argc < 3 || napi_get_value_external(env, argv[0], &ctx) != napi_ok ||
      napi_get_value_external(env, argv[1], &key) != napi_ok ||
      napi_get_buffer_info(env, argv[2], &wt, &wlen) != napi_ok) {
    napi_throw_type_error(env, nullptr, "prove(ctx, key, wtnsBuffer[, rsBuffer])");
    return nullptr;
  }
  ProveWork* w = new ProveWork();
  w->ctx = ctx_arg(env, argv[0]);  // throws the context's creation error
  if (!w->ctx) {
    delete w;
    return nullptr;
  }
  w->key = static_cast<zkfl_key*>(key);
  w->wtns.assign(static_cast<uint8_t*>(wt), static_cast<uint8_t*>(wt) + wlen);
  if (argc >= 4 && napi_get_buffer_info(env, argv[3], &rs, &rslen) == napi_ok && rslen == 64)
    w->rs.assign(static_cast<uint8_t*>(rs), static_cast<uint8_t*>(rs) + 64);
  napi_value promise, name;
  napi_create_promise(env, &w->deferred, &promise);
  napi_create_string_utf8(env, "zkfl_prove", NAPI_AUTO_LENGTH, &name);
  napi_create_async_work(env, nullptr, name, prove_execute, prove_complete, w, &w->work);
  napi_queue_async_work(env, w->work);
  return promise;
}

struct VerifyWork {
  napi_async_work work = nullptr;
  napi_deferred deferred = nullptr;
  zkfl_ctx* ctx = nullptr;
  std::vector<uint8_t> vk, pub, proof;
  int rc = 0;
  std::string err;
};

void verify_execute(napi_env, void* data) {
  VerifyWork* w = static_cast<VerifyWork*>(data);
  w->rc = zkfl_groth16_verify(w->ctx, w->vk.data(), w->vk.size(), w->pub.data(), w->pub.size() / 32,
                              w->proof.data());
  if (w->rc < 0) w->err = zkfl_last_error();
}

void verify_complete(napi_env env, napi_status, void* data) {
  VerifyWork* w = static_cast<VerifyWork*>(data);
  if (w->rc < 0) {
    napi_value msg, err;
    std::string m = "zkfl verify failed (" + std::to_string(w->rc) + "): " + w->err;
    napi_create_string_utf8(env, m.c_str(), NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, nullptr, msg, &err);
    napi_reject_deferred(env, w->deferred, err);
  } else {
    napi_value b;
    napi_get_boolean(env, w->rc == 1, &b);
    napi_resolve_deferred(env, w->deferred, b);
  }
  napi_delete_async_work(env, w->work);
  delete w;
}

napi_value Verify(napi_env env, napi_callback_info info) {
  size_t argc = 4;
  napi_value argv[4];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  void *ctx = nullptr, *vk = nullptr, *pub = nullptr, *pr = nullptr;
  size_t vlen = 0, plen = 0, prlen = 0;
  if (argc < 4 || napi_get_value_external(env, argv[0], &ctx) != napi_ok ||
      napi_get_buffer_info(env, argv[1], &vk, &vlen) != napi_ok ||
      napi_get_buffer_info(env, argv[2], &pub, &plen) != napi_ok ||
      napi_get_buffer_info(env, argv[3], &pr, &prlen) != napi_ok || prlen != 256 || plen % 32) {
    napi_throw_type_error(env, nullptr, "verify(ctx, vkBuffer, publicBuffer(n x 32), proofBuffer(256))");
    return nullptr;
  }
  VerifyWork* w = new VerifyWork();
  w->ctx = ctx_arg(env, argv[0]);  // throws the context's creation error
  if (!w->ctx) {
    delete w;
    return nullptr;
  }
  w->vk.assign(static_cast<uint8_t*>(vk), static_cast<uint8_t*>(vk) + vlen);
  w->pub.assign(static_cast<uint8_t*>(pub), static_cast<uint8_t*>(pub) + plen);
  w->pub.resize(plen + 32);  // never empty (data() of an empty vector may be null)
  w->pub.resize(plen);
  w->proof.assign(static_cast<uint8_t*>(pr), static_cast<uint8_t*>(pr) + 256);
  napi_value promise, name;
  napi_create_promise(env, &w->deferred, &promise);
  napi_create_string_utf8(env, "zkfl_verify", NAPI_AUTO_LENGTH, &name);
  napi_create_async_work(env, nullptr, name, verify_execute, verify_complete, w, &w->work);
  napi_queue_async_work(env, w->work);
  return promise;
}

napi_value LoadProgram(napi_env env, napi_callback_info info) {
  size_t argc = 2;
  napi_value argv[2];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  void* ctx = nullptr;
  void* data = nullptr;
  size_t len = 0;
  if (argc < 2 || napi_get_value_external(env, argv[0], &ctx) != napi_ok ||
      napi_get_buffer_info(env, argv[1], &data, &len) != napi_ok) {
    napi_throw_type_error(env, nullptr, "loadProgram(ctx, zkwpBuffer)");
    return nullptr;
  }
  zkfl_ctx* c = ctx_arg(env, argv[0]);
  if (!c) return nullptr;
  zkfl_wprog* prog = nullptr;
  int rc = zkfl_wprog_load(c, static_cast<const uint8_t*>(data), len, &prog);
  if (rc) return throw_err(env, rc);
  napi_value ext;
  napi_create_external(env, prog, prog_finalize, nullptr, &ext);
  return ext;
}

struct WitnessWork {
  napi_async_work work = nullptr;
  napi_deferred deferred = nullptr;
  zkfl_ctx* ctx = nullptr;
  zkfl_wprog* prog = nullptr;
  std::string json;
  std::vector<uint8_t> wtns;
  int rc = 0;
  std::string err;
};

void witness_execute(napi_env, void* data) {
  WitnessWork* w = static_cast<WitnessWork*>(data);
  w->wtns.resize(zkfl_wtns_size(w->prog));
  w->rc = zkfl_witness_compute_json(w->ctx, w->prog, w->json.c_str(), w->wtns.data());
  if (w->rc) w->err = zkfl_last_error();
}

void witness_complete(napi_env env, napi_status, void* data) {
  WitnessWork* w = static_cast<WitnessWork*>(data);
  if (w->rc) {
    napi_value msg, err;
    std::string m = "zkfl witness failed (" + std::to_string(w->rc) + "): " + w->err;
    napi_create_string_utf8(env, m.c_str(), NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, nullptr, msg, &err);
    napi_reject_deferred(env, w->deferred, err);
  } else {
    napi_value buf;
    void* p;
    napi_create_buffer_copy(env, w->wtns.size(), w->wtns.data(), &p, &buf);
    napi_resolve_deferred(env, w->deferred, buf);
  }
  napi_delete_async_work(env, w->work);
  delete w;
}

napi_value Witness(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  void *ctx = nullptr, *prog = nullptr;
  size_t jlen = 0;
  if (argc < 3 || napi_get_value_external(env, argv[0], &ctx) != napi_ok ||
      napi_get_value_external(env, argv[1], &prog) != napi_ok ||
      napi_get_value_string_utf8(env, argv[2], nullptr, 0, &jlen) != napi_ok) {
    napi_throw_type_error(env, nullptr, "witness(ctx, prog, inputJsonString)");
    return nullptr;
  }
  WitnessWork* w = new WitnessWork();
  w->ctx = ctx_arg(env, argv[0]);  // throws the context's creation error
  if (!w->ctx) {
    delete w;
    return nullptr;
  }
  w->prog = static_cast<zkfl_wprog*>(prog);
  w->json.resize(jlen + 1);
  napi_get_value_string_utf8(env, argv[2], &w->json[0], jlen + 1, &jlen);
  w->json.resize(jlen);
  napi_value promise, name;
  napi_create_promise(env, &w->deferred, &promise);
  napi_create_string_utf8(env, "zkfl_witness", NAPI_AUTO_LENGTH, &name);
  napi_create_async_work(env, nullptr, name, witness_execute, witness_complete, w, &w->work);
  napi_queue_async_work(env, w->work);
  return promise;
}

// snarkjs groth16.fullProve: input.json -> witness on the GPU -> proof, one call (the witness never
// leaves the device; tests/full_system_simulation.mjs:758-776 as two child processes in the reference)
struct FullProveWork {
  napi_async_work work = nullptr;
  napi_deferred deferred = nullptr;
  zkfl_ctx* ctx = nullptr;
  zkfl_key* key = nullptr;
  zkfl_wprog* prog = nullptr;
  std::string json;
  std::vector<uint8_t> rs, pub;
  uint8_t proof[256];
  uint32_t npub = 0;
  int rc = 0;
  std::string err;
};

void full_prove_execute(napi_env, void* data) {
  FullProveWork* w = static_cast<FullProveWork*>(data);
  uint32_t nv = 0, dom = 0;
  zkfl_key_info(w->key, &nv, &w->npub, &dom);
  w->pub.resize((size_t)w->npub * 32 + 32);
  w->rc = zkfl_groth16_full_prove_json(w->ctx, w->key, w->prog, w->json.c_str(), w->rs.empty() ? nullptr : w->rs.data(),
                                       w->proof, w->pub.data());
  if (w->rc) w->err = zkfl_last_error();
}

void full_prove_complete(napi_env env, napi_status, void* data) {
  FullProveWork* w = static_cast<FullProveWork*>(data);
  if (w->rc) {
    napi_value msg, err;
    std::string m = "zkfl fullProve failed (" + std::to_string(w->rc) + "): " + w->err;
    napi_create_string_utf8(env, m.c_str(), NAPI_AUTO_LENGTH, &msg);
    napi_create_error(env, nullptr, msg, &err);
    napi_reject_deferred(env, w->deferred, err);
  } else {
    napi_value obj, proof, pub;
    void* p;
    napi_create_buffer_copy(env, 256, w->proof, &p, &proof);
    napi_create_buffer_copy(env, (size_t)w->npub * 32, w->pub.data(), &p, &pub);
    napi_create_object(env, &obj);
    napi_set_named_property(env, obj, "proof", proof);
    napi_set_named_property(env, obj, "publicSignals", pub);
    napi_resolve_deferred(env, w->deferred, obj);
  }
  napi_delete_async_work(env, w->work);
  delete w;
}

napi_value FullProve(napi_env env, napi_callback_info info) {
  size_t argc = 5;
  napi_value argv[5];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  void *ctx = nullptr, *key = nullptr, *prog = nullptr, *rs = nullptr;
  size_t jlen = 0, rslen = 0;
  if (argc < 4 || napi_get_value_external(env, argv[0], &ctx) != napi_ok ||
      napi_get_value_external(env, argv[1], &key) != napi_ok ||
      napi_get_value_external(env, argv[2], &prog) != napi_ok ||
      napi_get_value_string_utf8(env, argv[3], nullptr, 0, &jlen) != napi_ok) {
    napi_throw_type_error(env, nullptr, "fullProve(ctx, key, prog, inputJsonString[, rsBuffer])");
    return nullptr;
  }
  FullProveWork* w = new FullProveWork();
  w->ctx = ctx_arg(env, argv[0]);  // throws the context's creation error
  if (!w->ctx) {
    delete w;
    return nullptr;
  }
  w->key = static_cast<zkfl_key*>(key);
  w->prog = static_cast<zkfl_wprog*>(prog);
  w->json.resize(jlen + 1);
  napi_get_value_string_utf8(env, argv[3], &w->json[0], jlen + 1, &jlen);
  w->json.resize(jlen);
  if (argc >= 5 && napi_get_buffer_info(env, argv[4], &rs, &rslen) == napi_ok && rslen == 64)
    w->rs.assign(static_cast<uint8_t*>(rs), static_cast<uint8_t*>(rs) + 64);
  napi_value promise, name;
  napi_create_promise(env, &w->deferred, &promise);
  napi_create_string_utf8(env, "zkfl_full_prove", NAPI_AUTO_LENGTH, &name);
  napi_create_async_work(env, nullptr, name, full_prove_execute, full_prove_complete, w, &w->work);
  napi_queue_async_work(env, w->work);
  return promise;
}

napi_value Pairing(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  void *ctx = nullptr, *g1 = nullptr, *g2 = nullptr;
  size_t l1 = 0, l2 = 0;
  if (argc < 3 || napi_get_value_external(env, argv[0], &ctx) != napi_ok ||
      napi_get_buffer_info(env, argv[1], &g1, &l1) != napi_ok || napi_get_buffer_info(env, argv[2], &g2, &l2) != napi_ok ||
      l1 != 64 || l2 != 128) {
    napi_throw_type_error(env, nullptr, "pairing(ctx, g1Buffer(64), g2Buffer(128))");
    return nullptr;
  }
  zkfl_ctx* c = ctx_arg(env, argv[0]);
  if (!c) return nullptr;
  uint8_t gt[384];
  int rc = zkfl_pairing(c, 1, static_cast<const uint8_t*>(g1),
                        static_cast<const uint8_t*>(g2), gt);
  if (rc) return throw_err(env, rc);
  napi_value buf;
  void* p;
  napi_create_buffer_copy(env, 384, gt, &p, &buf);
  return buf;
}

// Poseidon / vectorHash / Merkle trees on the GPU for the circomlibjs face (node/circomlibjs):
// the harness's off-circuit commitments (tests/full_system_simulation.mjs:134-238).  Synchronous:
// one small launch each, like circomlibjs's own synchronous `poseidon(...)`.
//   poseidon(ctx, arity, n, inputs(n*arity*32)) -> Buffer(n*32)          (zkfl_poseidon_batch)
//   vectorHash(ctx, len, n, values(n*len*32)) -> Buffer(n*32)            (zkfl_vector_hash_batch)
//   merkleBuild(ctx, leaves(n*32), depth) -> Buffer((2^(depth+1)-1)*32)  (zkfl_merkle_build)
bool get_ctx_buf(napi_env env, napi_value* argv, size_t argc, size_t need, void** ctx, void** data, size_t* len,
                 size_t buf_arg) {
  return argc >= need && napi_get_value_external(env, argv[0], ctx) == napi_ok &&
         napi_get_buffer_info(env, argv[buf_arg], data, len) == napi_ok;
}

napi_value HashCall(napi_env env, napi_callback_info info, bool vector) {
  size_t argc = 4;
  napi_value argv[4];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  void *ctx = nullptr, *in = nullptr;
  size_t len = 0;
  uint32_t width = 0, n = 0;
  if (!get_ctx_buf(env, argv, argc, 4, &ctx, &in, &len, 3) || napi_get_value_uint32(env, argv[1], &width) != napi_ok ||
      napi_get_value_uint32(env, argv[2], &n) != napi_ok || len != (size_t)width * n * 32) {
    napi_throw_type_error(env, nullptr, vector ? "vectorHash(ctx, len, n, valuesBuffer(n*len*32))"
                                               : "poseidon(ctx, arity, n, inputsBuffer(n*arity*32))");
    return nullptr;
  }
  zkfl_ctx* c = ctx_arg(env, argv[0]);
  if (!c) return nullptr;
  std::vector<uint8_t> out((size_t)n * 32 + 32);
  int rc = vector ? zkfl_vector_hash_batch(c, width, n, static_cast<const uint8_t*>(in), out.data())
                  : zkfl_poseidon_batch(c, width, n, static_cast<const uint8_t*>(in), out.data());
  if (rc) return throw_err(env, rc);
  napi_value buf;
  void* p;
  napi_create_buffer_copy(env, (size_t)n * 32, out.data(), &p, &buf);
  return buf;
}

napi_value Poseidon(napi_env env, napi_callback_info info) { return HashCall(env, info, false); }
napi_value VectorHash(napi_env env, napi_callback_info info) { return HashCall(env, info, true); }

napi_value MerkleBuild(napi_env env, napi_callback_info info) {
  size_t argc = 3;
  napi_value argv[3];
  napi_get_cb_info(env, info, &argc, argv, nullptr, nullptr);
  void *ctx = nullptr, *in = nullptr;
  size_t len = 0;
  uint32_t depth = 0;
  if (!get_ctx_buf(env, argv, argc, 3, &ctx, &in, &len, 1) || napi_get_value_uint32(env, argv[2], &depth) != napi_ok ||
      len % 32 || depth > ZKFL_MERKLE_MAX_DEPTH) {
    napi_throw_type_error(env, nullptr, "merkleBuild(ctx, leavesBuffer(n*32), depth)");
    return nullptr;
  }
  const size_t nodes = ((size_t)2 << depth) - 1;
  zkfl_ctx* c = ctx_arg(env, argv[0]);
  if (!c) return nullptr;
  std::vector<uint8_t> out(nodes * 32);
  int rc = zkfl_merkle_build(c, static_cast<const uint8_t*>(in), len / 32, depth, out.data());
  if (rc) return throw_err(env, rc);
  napi_value buf;
  void* p;
  napi_create_buffer_copy(env, out.size(), out.data(), &p, &buf);
  return buf;
}

napi_value Init(napi_env env, napi_value exports) {
  napi_property_descriptor props[] = {
      {"version", nullptr, Version, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"deviceCount", nullptr, DeviceCount, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"createContext", nullptr, CreateContext, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"loadKey", nullptr, LoadKey, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"openKeyFile", nullptr, OpenKeyFile, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"loadKeyFile", nullptr, LoadKeyFile, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"contextReady", nullptr, ContextReady, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"quickExit", nullptr, QuickExit, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"keyInfo", nullptr, KeyInfo, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"prove", nullptr, Prove, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"verify", nullptr, Verify, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"loadProgram", nullptr, LoadProgram, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"witness", nullptr, Witness, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"fullProve", nullptr, FullProve, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"pairing", nullptr, Pairing, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"poseidon", nullptr, Poseidon, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"vectorHash", nullptr, VectorHash, nullptr, nullptr, nullptr, napi_default, nullptr},
      {"merkleBuild", nullptr, MerkleBuild, nullptr, nullptr, nullptr, napi_default, nullptr},
  };
  napi_define_properties(env, exports, sizeof(props) / sizeof(props[0]), props);
  return exports;
}

}  // namespace

NAPI_MODULE(NODE_GYP_MODULE_NAME, Init)
