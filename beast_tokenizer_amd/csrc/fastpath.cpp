// Host fast path for BEASTBsplineTokenizer.encode / reconstruct_traj (default time grid), and
// the List[List[int]] builder of the BPE tokenizer's encode (rows_to_lists).
//
// Host-side C++ only: the same C-ABI entry points the ctypes binding calls
// (beast_encode_f32 / beast_reconstruct_f32 in libbeast_hip.so, passed in as function
// pointers so this module does not link the library), with the output tensors allocated by
// ATen instead of through Python.  It saves the per-call Python cost of two torch.empty and
// the ctypes argument marshalling (the B=4096 step is host-bound).  Anything
// unusual (non-contiguous input, wrong device / dtype / shape) returns None and the caller
// takes the general Python path, which raises the reference's exception types.
#include <torch/extension.h>
#include <torch/csrc/autograd/python_variable.h>
#include <c10/hip/HIPStream.h>

#include <algorithm>
#include <chrono>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

namespace {

typedef int (*enc_fn_t)(const float*, int64_t, int, int64_t, int64_t, int64_t, int, int, int, const int32_t*,
                        const float*, int, const float*, const float*, int, int64_t, float*, int64_t*, void*);
typedef int (*rec_fn_t)(const int64_t*, int64_t, int, int, int, int, int64_t, const float*, const float*,
                        const float*, int64_t, int, const int32_t*, int, const float*, int64_t, const int32_t*, float*,
                        float*, const float*, void*);
typedef const char* (*err_fn_t)(void);

// tokens int64 [B, DN] and params fp32 [B, DN] as two tensors over ONE caching-allocator block
// (tokens first, params at byte 8*B*DN): one allocator round trip per encode instead of two
// (the B = 4,096 step is at the host / GPU crossover).  Each tensor is a plain
// TensorImpl over the shared storage, sized directly -- no narrow / dtype-view chain.
inline void alloc_enc_outputs(const at::Tensor& like, int64_t B, int64_t DN, at::Tensor& tokens, at::Tensor& params) {
  const int64_t n = B * DN;
  at::Tensor buf = at::empty({n * 12}, like.options().dtype(at::kByte));
  const c10::Storage& st = buf.storage();
  tokens = at::detail::make_tensor<c10::TensorImpl>(c10::Storage(st), buf.key_set(),
                                                     caffe2::TypeMeta::Make<int64_t>());
  const int64_t sz[2] = {B, DN}, sd[2] = {DN, 1};
  tokens.unsafeGetTensorImpl()->set_sizes_and_strides(c10::IntArrayRef(sz, 2), c10::IntArrayRef(sd, 2),
                                                      std::optional<int64_t>(0));
  params = at::detail::make_tensor<c10::TensorImpl>(c10::Storage(st), buf.key_set(), caffe2::TypeMeta::Make<float>());
  params.unsafeGetTensorImpl()->set_sizes_and_strides(c10::IntArrayRef(sz, 2), c10::IntArrayRef(sd, 2),
                                                      std::optional<int64_t>(2 * n));   // offset in floats
}

struct Plan {
  enc_fn_t enc = nullptr;
  rec_fn_t rec = nullptr;
  err_fn_t err = nullptr;
  int64_t device = 0;
  int64_t D = 0, nj = 0, N = 0, T = 0, V = 0, min_din = 0;
  int64_t p_src = 0, p_proj = 0, p_wmn = 0, p_wmx = 0, p_phi = 0, p_dst = 0;

  void fail(int rc, const char* what) const {
    std::string m = std::string(what) + ": " + (err ? err() : "error") + " (code " + std::to_string(rc) + ")";
    throw std::runtime_error(m);
  }

  // (tokens int64 [B, N*D] + offset, params fp32 [B, D*N]) or None
  py::object encode(const at::Tensor& x, int64_t offset, int64_t stream) const {
    if (!x.is_cuda() || x.get_device() != device || x.scalar_type() != at::kFloat || x.dim() != 3 ||
        x.size(1) != T || x.size(2) < min_din || x.stride(2) != 1)
      return py::none();
    const int64_t B = x.size(0);
    const int64_t DN = D * N;
    at::Tensor params = at::empty({B, DN}, x.options());
    at::Tensor tokens = at::empty({B, DN}, x.options().dtype(at::kLong));
    const int rc = enc(x.data_ptr<float>(), B, (int)T, x.stride(0), x.stride(1), x.stride(2), (int)x.size(2), (int)D,
                       (int)nj, reinterpret_cast<const int32_t*>(p_src), reinterpret_cast<const float*>(p_proj),
                       (int)N, reinterpret_cast<const float*>(p_wmn), reinterpret_cast<const float*>(p_wmx), (int)V,
                       offset, params.data_ptr<float>(), tokens.data_ptr<int64_t>(),
                       reinterpret_cast<void*>(stream));
    if (rc) fail(rc, "beast_encode_f32");
    return py::make_tuple(tokens, params);
  }

  // params fp32 [B, D*N] only (compute_weights / fit_parameters) or None
  py::object fit(const at::Tensor& x, int64_t stream) const {
    if (!x.is_cuda() || x.get_device() != device || x.scalar_type() != at::kFloat || x.dim() != 3 ||
        x.size(1) != T || x.size(2) < min_din || x.stride(2) != 1)
      return py::none();
    const int64_t B = x.size(0);
    at::Tensor params = at::empty({B, D * N}, x.options());
    const int rc = enc(x.data_ptr<float>(), B, (int)T, x.stride(0), x.stride(1), x.stride(2), (int)x.size(2), (int)D,
                       (int)nj, reinterpret_cast<const int32_t*>(p_src), reinterpret_cast<const float*>(p_proj),
                       (int)N, nullptr, nullptr, (int)V, 0, params.data_ptr<float>(), nullptr,
                       reinterpret_cast<void*>(stream));
    if (rc) fail(rc, "beast_encode_f32");
    return py::cast(params);
  }

  // positions fp32 [B, T, D] from int64 tokens [B, N*D] (or [B, N, D]) or None
  py::object reconstruct(const at::Tensor& tok, int64_t offset, int64_t stream) const {
    if (!tok.is_cuda() || tok.get_device() != device || tok.scalar_type() != at::kLong || !tok.is_contiguous())
      return py::none();
    const int64_t DN = D * N;
    int64_t B;
    if (tok.dim() == 2 && tok.size(1) == DN) B = tok.size(0);
    else if (tok.dim() == 3 && tok.size(1) * tok.size(2) == DN) B = tok.size(0);
    else return py::none();
    at::Tensor pos = at::empty({B, T, D}, tok.options().dtype(at::kFloat));
    const int rc = rec(tok.data_ptr<int64_t>(), B, (int)D, (int)nj, (int)N, (int)V, offset,
                       reinterpret_cast<const float*>(p_wmn), reinterpret_cast<const float*>(p_wmx),
                       reinterpret_cast<const float*>(p_phi), 0, (int)T, reinterpret_cast<const int32_t*>(p_dst),
                       (int)D, nullptr, 0, nullptr, nullptr, pos.data_ptr<float>(), nullptr,
                       reinterpret_cast<void*>(stream));
    if (rc) fail(rc, "beast_reconstruct_f32");
    return py::cast(pos);
  }

  // Diagnostic (tools/host_split.py): host microseconds per call of the pieces of encode, over n
  // back-to-back calls each -- the two output allocations, the C-ABI call with preallocated
  // outputs (validation + launch), and the whole fast-path call.
  py::dict time_parts(const at::Tensor& x, int64_t stream, int64_t n) const {
    using clk = std::chrono::steady_clock;
    auto us = [&](clk::time_point t0) { return std::chrono::duration<double, std::micro>(clk::now() - t0).count() / n; };
    const int64_t B = x.size(0), DN = D * N;
    py::dict out;
    auto t0 = clk::now();
    for (int64_t i = 0; i < n; ++i) {
      at::Tensor p = at::empty({B, DN}, x.options());
      at::Tensor t = at::empty({B, DN}, x.options().dtype(at::kLong));
    }
    out["alloc2"] = us(t0);
    t0 = clk::now();
    for (int64_t i = 0; i < n; ++i) {
      at::Tensor p, t;
      alloc_enc_outputs(x, B, DN, t, p);
    }
    out["alloc1_shared"] = us(t0);
    at::Tensor params = at::empty({B, DN}, x.options());
    at::Tensor tokens = at::empty({B, DN}, x.options().dtype(at::kLong));
    t0 = clk::now();
    for (int64_t i = 0; i < n; ++i)
      enc(x.data_ptr<float>(), B, (int)T, x.stride(0), x.stride(1), x.stride(2), (int)x.size(2), (int)D, (int)nj,
          reinterpret_cast<const int32_t*>(p_src), reinterpret_cast<const float*>(p_proj), (int)N,
          reinterpret_cast<const float*>(p_wmn), reinterpret_cast<const float*>(p_wmx), (int)V, 0,
          params.data_ptr<float>(), tokens.data_ptr<int64_t>(), reinterpret_cast<void*>(stream));
    out["abi_call"] = us(t0);
    t0 = clk::now();
    for (int64_t i = 0; i < n; ++i) encode(x, 0, stream);
    out["fast_encode_cpp"] = us(t0);
    return out;
  }
};

Plan make_plan(int64_t enc, int64_t rec, int64_t err, int64_t device, int64_t D, int64_t nj, int64_t N, int64_t T,
               int64_t V, int64_t min_din, int64_t p_src, int64_t p_proj, int64_t p_wmn, int64_t p_wmx, int64_t p_phi,
               int64_t p_dst) {
  Plan p;
  p.enc = reinterpret_cast<enc_fn_t>(enc);
  p.rec = reinterpret_cast<rec_fn_t>(rec);
  p.err = reinterpret_cast<err_fn_t>(err);
  p.device = device;
  p.D = D; p.nj = nj; p.N = N; p.T = T; p.V = V; p.min_din = min_din;
  p.p_src = p_src; p.p_proj = p_proj; p.p_wmn = p_wmn; p.p_wmx = p_wmx; p.p_phi = p_phi; p.p_dst = p_dst;
  if (!p.enc || !p.rec || !p.err) throw std::invalid_argument("null entry point");
  return p;
}

// BPE encode's result as the reference returns it, List[List[int]] (beast_bspline_bpe_tokenizer.py
// :175-199 builds one list per row from HF's ids): rows ids[r, :lens[r]] of a host int32 [R, W]
// tensor.  The per-element cost of building Python ints dominates the list comprehension, so ids
// below 65,536 share one cached int object each (ints are immutable; each slot holds a reference).
py::list rows_to_lists(const at::Tensor& ids, const at::Tensor& lens) {
  if (ids.is_cuda() || lens.is_cuda() || ids.scalar_type() != at::kInt || lens.scalar_type() != at::kInt ||
      ids.dim() != 2 || lens.dim() != 1 || lens.size(0) != ids.size(0) || !ids.is_contiguous() ||
      !lens.is_contiguous())
    throw std::invalid_argument("rows_to_lists: host int32 ids [R, W] and lens [R] expected");
  static std::vector<PyObject*> cache;
  if (cache.empty()) {
    cache.resize(65536);
    for (int i = 0; i < 65536; ++i) cache[i] = PyLong_FromLong(i);   // held for the process lifetime
  }
  const int64_t R = ids.size(0), W = ids.size(1);
  const int32_t* p = ids.data_ptr<int32_t>();
  const int32_t* L = lens.data_ptr<int32_t>();
  // thousands of fresh lists would trigger generation-0 collections that traverse them again and
  // again (measured 2.4x the build time); the collector is paused for the build and restored
  struct GcPause {
    int was = PyGC_Disable();
    ~GcPause() { if (was) PyGC_Enable(); }
  } gc_pause;
  // every list slot holds a reference to a cached int: instead of one Py_INCREF per slot (a
  // read-modify-write of a refcount that the same few thousand objects keep repeating), count the
  // slots per id first and add each id's count to its refcount once
  std::vector<Py_ssize_t> uses(65536, 0);   // per call: nothing stale survives a throw
  int32_t hi = -1;
  for (int64_t r = 0; r < R; ++r) {
    const int64_t n = std::min<int64_t>(std::max<int32_t>(L[r], 0), W);
    const int32_t* q = p + r * W;
    for (int64_t i = 0; i < n; ++i) {
      const int32_t v = q[i];
      if (v >= 0 && v < 65536) { ++uses[v]; hi = std::max(hi, v); }
    }
  }
  for (int32_t v = 0; v <= hi; ++v)
    if (uses[v]) { Py_SET_REFCNT(cache[v], Py_REFCNT(cache[v]) + uses[v]); uses[v] = 0; }
  // on an allocation failure the references counted for slots never filled (row r from slot i on,
  // and every later row) are handed back before the throw
  auto fail = [&](int64_t r, int64_t i, PyObject* row, PyObject* out) {
    for (int64_t rr = r; rr < R; ++rr) {
      const int64_t n = std::min<int64_t>(std::max<int32_t>(L[rr], 0), W);
      const int32_t* q = p + rr * W;
      for (int64_t k = rr == r ? i : 0; k < n; ++k)
        if (q[k] >= 0 && q[k] < 65536) Py_DECREF(cache[q[k]]);
    }
    Py_XDECREF(row);   // drops the slots it holds (a fresh list's empty slots are NULL)
    Py_XDECREF(out);
    throw py::error_already_set();
  };
  PyObject* out = PyList_New(R);
  if (!out) fail(0, 0, nullptr, nullptr);
  for (int64_t r = 0; r < R; ++r) {
    const int64_t n = std::min<int64_t>(std::max<int32_t>(L[r], 0), W);
    PyObject* row = PyList_New(n);
    if (!row) fail(r, 0, nullptr, out);
    const int32_t* q = p + r * W;
    for (int64_t i = 0; i < n; ++i) {
      const int32_t v = q[i];
      PyObject* o;
      if (v >= 0 && v < 65536) o = cache[v];   // its reference was counted above
      else if (!(o = PyLong_FromLong(v))) fail(r, i, row, out);
      PyList_SET_ITEM(row, i, o);
    }
    PyList_SET_ITEM(out, r, row);
  }
  return py::reinterpret_steal<py::list>(out);
}

// The per-call entry points as CPython METH_FASTCALL functions: (plan address, tensor, offset),
// the current stream of the plan's device taken here, the reference's return value built here
// (encode: (tokens, params dict)).  A pybind11 method call, the Python-side stream query and
// the dict / tuple building cost about as much host time as the C-ABI call's own validation.
PyObject* g_keys[5] = {};   // "params", "init_pos", "init_vel", "end_pos", "end_vel"

inline const Plan* plan_of(PyObject* addr) { return reinterpret_cast<const Plan*>(PyLong_AsVoidPtr(addr)); }

PyObject* fast_encode(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "fast_encode(plan, x, offset)");
    return nullptr;
  }
  const Plan* p = plan_of(args[0]);
  const long long offset = PyLong_AsLongLong(args[2]);
  if ((p == nullptr || offset == -1) && PyErr_Occurred()) return nullptr;
  if (!THPVariable_Check(args[1])) Py_RETURN_NONE;
  const at::Tensor& x = THPVariable_Unpack(args[1]);
  if (!x.is_cuda() || x.get_device() != p->device || x.scalar_type() != at::kFloat || x.dim() != 3 ||
      x.size(1) != p->T || x.size(2) < p->min_din || x.stride(2) != 1)
    Py_RETURN_NONE;
  at::Tensor params, tokens;
  try {
    const int64_t B = x.size(0), DN = p->D * p->N;
    alloc_enc_outputs(x, B, DN, tokens, params);
    const hipStream_t st = c10::hip::getCurrentHIPStream(p->device).stream();
    const int rc = p->enc(x.data_ptr<float>(), B, (int)p->T, x.stride(0), x.stride(1), x.stride(2), (int)x.size(2),
                          (int)p->D, (int)p->nj, reinterpret_cast<const int32_t*>(p->p_src),
                          reinterpret_cast<const float*>(p->p_proj), (int)p->N,
                          reinterpret_cast<const float*>(p->p_wmn), reinterpret_cast<const float*>(p->p_wmx),
                          (int)p->V, offset, params.data_ptr<float>(), tokens.data_ptr<int64_t>(),
                          reinterpret_cast<void*>(st));
    if (rc) p->fail(rc, "beast_encode_f32");
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
  PyObject* d = PyDict_New();
  PyObject* po = THPVariable_Wrap(std::move(params));
  PyObject* to = THPVariable_Wrap(std::move(tokens));
  if (!d || !po || !to || PyDict_SetItem(d, g_keys[0], po) < 0) {
    Py_XDECREF(d); Py_XDECREF(po); Py_XDECREF(to);
    return nullptr;
  }
  Py_DECREF(po);
  for (int i = 1; i < 5; ++i)
    if (PyDict_SetItem(d, g_keys[i], Py_None) < 0) {
      Py_DECREF(d); Py_DECREF(to);
      return nullptr;
    }
  PyObject* r = PyTuple_New(2);
  if (!r) { Py_DECREF(d); Py_DECREF(to); return nullptr; }
  PyTuple_SET_ITEM(r, 0, to);
  PyTuple_SET_ITEM(r, 1, d);
  return r;
}

PyObject* fast_reconstruct(PyObject*, PyObject* const* args, Py_ssize_t nargs) {
  if (nargs != 3) {
    PyErr_SetString(PyExc_TypeError, "fast_reconstruct(plan, tokens, offset)");
    return nullptr;
  }
  const Plan* p = plan_of(args[0]);
  const long long offset = PyLong_AsLongLong(args[2]);
  if ((p == nullptr || offset == -1) && PyErr_Occurred()) return nullptr;
  if (!THPVariable_Check(args[1])) Py_RETURN_NONE;
  const at::Tensor& tok = THPVariable_Unpack(args[1]);
  if (!tok.is_cuda() || tok.get_device() != p->device || tok.scalar_type() != at::kLong || !tok.is_contiguous())
    Py_RETURN_NONE;
  const int64_t DN = p->D * p->N;
  int64_t B;
  if (tok.dim() == 2 && tok.size(1) == DN) B = tok.size(0);
  else if (tok.dim() == 3 && tok.size(1) * tok.size(2) == DN) B = tok.size(0);
  else Py_RETURN_NONE;
  at::Tensor pos;
  try {
    pos = at::empty({B, p->T, p->D}, tok.options().dtype(at::kFloat));
    const hipStream_t st = c10::hip::getCurrentHIPStream(p->device).stream();
    const int rc = p->rec(tok.data_ptr<int64_t>(), B, (int)p->D, (int)p->nj, (int)p->N, (int)p->V, offset,
                          reinterpret_cast<const float*>(p->p_wmn), reinterpret_cast<const float*>(p->p_wmx),
                          reinterpret_cast<const float*>(p->p_phi), 0, (int)p->T,
                          reinterpret_cast<const int32_t*>(p->p_dst), (int)p->D, nullptr, 0, nullptr, nullptr,
                          pos.data_ptr<float>(), nullptr, reinterpret_cast<void*>(st));
    if (rc) p->fail(rc, "beast_reconstruct_f32");
  } catch (const std::exception& e) {
    PyErr_SetString(PyExc_RuntimeError, e.what());
    return nullptr;
  }
  return THPVariable_Wrap(std::move(pos));
}

PyMethodDef g_fast_defs[] = {
    {"fast_encode", reinterpret_cast<PyCFunction>(reinterpret_cast<void*>(fast_encode)), METH_FASTCALL,
     "fast_encode(plan_addr, x, offset) -> (tokens, params dict) or None"},
    {"fast_reconstruct", reinterpret_cast<PyCFunction>(reinterpret_cast<void*>(fast_reconstruct)), METH_FASTCALL,
     "fast_reconstruct(plan_addr, tokens, offset) -> positions or None"},
};

}  // namespace


// The BPE trainer's log replay (bpe_train.train_bpe): for each logged merge (a, b, nid, reused) of
// the device loop, the new token's string id2str[a] + id2str[b] against the vocabulary -- an id the
// device re-used must be the string's, a new one must be the next id -- then the merge as a pair of
// strings.  id2str (list) and str2id (dict) are extended in place.  Returns the merges, or None at
// the first entry that disagrees (a 64-bit string-hash collision on the device: the caller reruns
// on the host-driven loop).  The same checks as the Python loop, ~10x faster (1,724 merges: the
// Python loop took ~2 ms of the K5 merge loop's wall time).
py::object replay_merge_log(py::list id2str, py::dict str2id, const at::Tensor& log) {
  if (log.is_cuda() || log.scalar_type() != at::kInt || log.dim() != 2 || (log.numel() && log.size(1) != 4) ||
      !log.is_contiguous())
    throw std::invalid_argument("replay_merge_log: host int32 log [n, 4] expected");
  const int64_t n = log.numel() ? log.size(0) : 0;
  const int32_t* L = log.data_ptr<int32_t>();
  PyObject* ids = id2str.ptr();
  PyObject* s2i = str2id.ptr();
  PyObject* merges = PyList_New(n);
  if (!merges) throw py::error_already_set();
  for (int64_t k = 0; k < n; ++k) {
    const int32_t a = L[4 * k], b = L[4 * k + 1], nid = L[4 * k + 2], reused = L[4 * k + 3];
    const Py_ssize_t nt = PyList_GET_SIZE(ids);
    if (a < 0 || b < 0 || a >= nt || b >= nt) { Py_DECREF(merges); return py::none(); }
    PyObject* sa = PyList_GET_ITEM(ids, a);   // borrowed
    PyObject* sb = PyList_GET_ITEM(ids, b);
    PyObject* tok = PyUnicode_Concat(sa, sb);
    if (!tok) { Py_DECREF(merges); throw py::error_already_set(); }
    PyObject* have = PyDict_GetItemWithError(s2i, tok);   // borrowed
    if (!have && PyErr_Occurred()) { Py_DECREF(tok); Py_DECREF(merges); throw py::error_already_set(); }
    const bool ok = have ? (reused && PyLong_AsLong(have) == nid) : (!reused && nid == nt);
    if (!ok) { Py_DECREF(tok); Py_DECREF(merges); return py::none(); }
    if (!have) {
      PyObject* id = PyLong_FromLong(nid);
      if (!id || PyDict_SetItem(s2i, tok, id) < 0 || PyList_Append(ids, tok) < 0) {
        Py_XDECREF(id); Py_DECREF(tok); Py_DECREF(merges);
        throw py::error_already_set();
      }
      Py_DECREF(id);
    }
    Py_DECREF(tok);
    PyObject* pair = PyTuple_Pack(2, sa, sb);
    if (!pair) { Py_DECREF(merges); throw py::error_already_set(); }
    PyList_SET_ITEM(merges, k, pair);
  }
  return py::reinterpret_steal<py::list>(merges);
}

PYBIND11_MODULE(TORCH_EXTENSION_NAME, m) {
  m.doc() = "host fast path of the BEAST encode / reconstruct calls (see csrc/fastpath.cpp)";
  py::class_<Plan>(m, "Plan")
      .def("encode", &Plan::encode, py::arg("x"), py::arg("offset"), py::arg("stream"))
      .def("fit", &Plan::fit, py::arg("x"), py::arg("stream"))
      .def("reconstruct", &Plan::reconstruct, py::arg("tokens"), py::arg("offset"), py::arg("stream"))
      .def("time_parts", &Plan::time_parts, py::arg("x"), py::arg("stream"), py::arg("n"))
      .def("addr", [](const Plan& p) { return reinterpret_cast<intptr_t>(&p); });
  m.def("make_plan", &make_plan);
  const char* keys[5] = {"params", "init_pos", "init_vel", "end_pos", "end_vel"};
  for (int i = 0; i < 5; ++i) g_keys[i] = PyUnicode_InternFromString(keys[i]);   // held for the process
  for (auto& def : g_fast_defs) {
    PyObject* f = PyCFunction_NewEx(&def, nullptr, m.ptr());
    if (!f) throw py::error_already_set();
    m.add_object(def.ml_name, py::reinterpret_steal<py::object>(f));
  }
  m.def("rows_to_lists", &rows_to_lists, py::arg("ids"), py::arg("lens"));
  m.def("replay_merge_log", &replay_merge_log, py::arg("id2str"), py::arg("str2id"), py::arg("log"));
}
