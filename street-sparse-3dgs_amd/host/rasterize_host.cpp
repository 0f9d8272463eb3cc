// rasterize_host.cpp -- the rasterizer's per-call host path as a compiled CPython extension
// (diff_gaussian_rasterization/_gsr_host.so), over the C ABI of libgsr_hip.so (include/gsr.h).
//
// The reference binds its CUDA rasterizer as a torch extension whose functions the autograd
// Function calls once per frame (diff_gaussian_rasterization/__init__.py of the hierarchy
// rasterizer; callers gaussian_renderer/__init__.py:105-113, 268-270, 391).  Round 4 did the same
// marshalling in Python over ctypes: argument validation, output allocation, three resize callbacks
// into Python, the autograd Function's forward / backward in Python (~0.26 ms of host time per
// fwd+bwd).  Here all of it is C++:
//
//   rasterize_gaussians(...)            = _C.rasterize_gaussians            (upstream signature)
//   rasterize_gaussians_backward(...)   = _C.rasterize_gaussians_backward   (upstream signature)
//   mark_visible(means3D, view, proj)   = _C.mark_visible
//   rasterize(means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3D_precomp,
//             raster_settings)          = _RasterizeGaussians.apply (a C++ autograd Function: its
//                                         backward runs on autograd's device thread without the GIL)
//
// Error behaviour follows the Python module it replaces (same messages; RuntimeError).  Scratch
// buffers are uint8 tensors from the torch caching allocator, made by C++ resize callbacks.
#include <torch/extension.h>
#include <torch/csrc/autograd/custom_function.h>
#include <c10/hip/HIPStream.h>

#include <dlfcn.h>

#include <atomic>
#include <mutex>
#include <string>

#include "gsr.h"

namespace py = pybind11;
using at::Tensor;
using torch::autograd::AutogradContext;
using torch::autograd::variable_list;

namespace {

[[noreturn]] void fail(const std::string &msg) { throw std::runtime_error(msg); }

// The C ABI entry points, bound at import from the library the ctypes layer loaded (bind(path): the
// same file, so the same library state; GSR_LIBRARY variants included).
struct Abi {
    decltype(&gsr_rasterize_forward_ex) forward_ex = nullptr;
    decltype(&gsr_rasterize_backward) backward = nullptr;
    decltype(&gsr_mark_visible) mark_visible = nullptr;
    decltype(&gsr_last_error) last_error = nullptr;
    decltype(&gsr_abi_version) abi_version = nullptr;
} g_abi;

const Abi &abi() {
    if (!g_abi.forward_ex) fail("diff_gaussian_rasterization: the host extension is not bound to libgsr_hip.so");
    return g_abi;
}

int bind(const std::string &path) {
    void *h = dlopen(path.c_str(), RTLD_NOW | RTLD_LOCAL);
    if (!h) fail(std::string("cannot load ") + path + ": " + dlerror());
    Abi a;
    a.forward_ex = reinterpret_cast<decltype(a.forward_ex)>(dlsym(h, "gsr_rasterize_forward_ex"));
    a.backward = reinterpret_cast<decltype(a.backward)>(dlsym(h, "gsr_rasterize_backward"));
    a.mark_visible = reinterpret_cast<decltype(a.mark_visible)>(dlsym(h, "gsr_mark_visible"));
    a.last_error = reinterpret_cast<decltype(a.last_error)>(dlsym(h, "gsr_last_error"));
    a.abi_version = reinterpret_cast<decltype(a.abi_version)>(dlsym(h, "gsr_abi_version"));
    if (!a.forward_ex || !a.backward || !a.mark_visible || !a.last_error || !a.abi_version)
        fail(path + " does not export the rasterizer's C ABI");
    if (a.abi_version() != GSR_ABI_VERSION) fail(path + ": ABI version mismatch; rebuild it");
    g_abi = a;
    return a.abi_version();
}

std::string dtype_name(at::ScalarType t) {
    switch (t) {
        case at::kFloat: return "torch.float32";
        case at::kDouble: return "torch.float64";
        case at::kHalf: return "torch.float16";
        case at::kBFloat16: return "torch.bfloat16";
        case at::kInt: return "torch.int32";
        case at::kLong: return "torch.int64";
        case at::kByte: return "torch.uint8";
        case at::kBool: return "torch.bool";
        default: return std::string("torch.") + c10::toString(t);
    }
}

bool present(const Tensor &t) { return t.defined() && t.numel() != 0; }

void require_gpu(const Tensor &t) {
    if (!t.defined() || !t.is_cuda())
        fail("diff_gaussian_rasterization (gfx950) requires tensors on a ROCm GPU device; there is no CPU path");
}

// _C.py _dev_f32: absent / empty -> undefined; else on `dev`, float32, contiguous
Tensor dev_f32(const Tensor &t, const char *name, const at::Device &dev) {
    if (!present(t)) return Tensor();
    if (t.device() != dev) fail(std::string(name) + " must be on " + dev.str() + " (got " + t.device().str() + ")");
    if (t.scalar_type() != at::kFloat)
        fail(std::string(name) + " must be float32 (got " + dtype_name(t.scalar_type()) + ")");
    return t.is_contiguous() ? t : t.contiguous();
}

Tensor saved(const Tensor &t) {  // a tensor the forward already validated
    if (!present(t)) return Tensor();
    return t.is_contiguous() ? t : t.contiguous();
}

template <class T>
T *ptr(const Tensor &t) {
    return present(t) ? static_cast<T *>(t.data_ptr()) : nullptr;
}
const float *fp(const Tensor &t) { return ptr<const float>(t); }
float *wp(const Tensor &t) { return ptr<float>(t); }

void check(int rc, const char *what) {
    if (rc != 0) fail(std::string(what) + " failed (" + std::to_string(rc) + "): " + abi().last_error());
}

void *stream_of(const at::Device &dev) { return c10::hip::getCurrentHIPStream(dev.index()).stream(); }

// ---- resize callbacks: uint8 tensors from the caching allocator --------------------------------
struct Buffers {
    at::TensorOptions opts;
    Tensor geom, binning, image, scratch;
    std::string err;
};
void *alloc_into(Buffers *b, Tensor &slot, size_t n) {
    try {
        slot = at::empty({(int64_t)std::max<size_t>(n, 1)}, b->opts);
        return slot.data_ptr();
    } catch (const std::exception &e) {  // the library reports GSR_ERR_ALLOCATION; the message is kept
        b->err = e.what();
        return nullptr;
    }
}
void *resize_geom(void *ctx, size_t n) { auto *b = static_cast<Buffers *>(ctx); return alloc_into(b, b->geom, n); }
void *resize_binning(void *ctx, size_t n) { auto *b = static_cast<Buffers *>(ctx); return alloc_into(b, b->binning, n); }
void *resize_image(void *ctx, size_t n) { auto *b = static_cast<Buffers *>(ctx); return alloc_into(b, b->image, n); }
void *resize_scratch(void *ctx, size_t n) { auto *b = static_cast<Buffers *>(ctx); return alloc_into(b, b->scratch, n); }

void check_call(int rc, const char *what, const Buffers &b) {
    if (rc != 0 && !b.err.empty())
        fail(std::string(what) + " failed (" + std::to_string(rc) + "): " + abi().last_error() + " [" + b.err + "]");
    check(rc, what);
}

Tensor u8_or_empty(const Tensor &t, const at::Device &dev) {
    return t.defined() ? t : at::empty({0}, at::TensorOptions().dtype(at::kByte).device(dev));
}

// ---- the hierarchy-cut fields (_C.py _cut_args) ------------------------------------------------
struct Cut {
    int n = 0;
    Tensor ri, pi, w, kids;
};
Cut cut_args(const Tensor &ri, const Tensor &pi, const Tensor &w, const Tensor &kids, const at::Device &dev) {
    Cut c;
    c.n = ri.defined() ? (int)ri.numel() : 0;
    if (c.n == 0) return c;
    if (!pi.defined() || !w.defined() || pi.numel() < c.n || w.numel() < c.n)
        fail("render_indices needs parent_indices and interpolation_weights of at least as many entries");
    auto i32 = [&](const Tensor &t) { return t.to(dev, at::kInt).contiguous(); };
    c.ri = i32(ri);
    c.pi = i32(pi);
    c.w = w.to(dev, at::kFloat).contiguous();
    if (kids.defined() && kids.numel()) c.kids = i32(kids);
    return c;
}

// one cached zero per device: the source of the zero-stride gradient views
Tensor zero_of(const at::Device &dev) {
    static std::mutex mu;
    static Tensor z[64];
    std::lock_guard<std::mutex> lk(mu);
    const int i = dev.index() < 0 ? 0 : dev.index() % 64;
    if (!z[i].defined()) z[i] = at::zeros({1}, at::TensorOptions().dtype(at::kFloat).device(dev));
    return z[i];
}

// gsr_dist.GradBucket: while a bucket captures a backward, the leaf gradients of means3D and the SH
// coefficients are written into views of its flat buffer (gsr_dist.grad_out).  The provider is set
// only for the capture (gsr_dist notifies), so an ordinary backward never takes the GIL.
// g_provider is read and written under the GIL only; g_provider_set is the GIL-free hint.
std::atomic<bool> g_provider_set{false};
PyObject *g_provider = nullptr;  // a new reference while set

// Releases the GIL for a library call when the calling thread holds it (the autograd engine's device
// thread runs the C++ backward without it).
struct NoGil {
    PyThreadState *st = nullptr;
    NoGil() {
        if (Py_IsInitialized() && PyGILState_Check()) st = PyEval_SaveThread();
    }
    ~NoGil() {
        if (st) PyEval_RestoreThread(st);
    }
};

Tensor leaf_grad(const Tensor &key, at::IntArrayRef shape, const at::Device &dev) {
    if (g_provider_set.load(std::memory_order_acquire)) {
        py::gil_scoped_acquire gil;
        if (!g_provider) return at::empty(shape, at::TensorOptions().dtype(at::kFloat).device(dev));
        py::object f = py::reinterpret_borrow<py::object>(g_provider);
        py::object k = key.defined() ? py::object(py::int_((uintptr_t)key.data_ptr())) : py::object(py::none());
        py::tuple shp(shape.size());
        for (size_t i = 0; i < shape.size(); i++) shp[i] = py::int_(shape[i]);
        py::object dv = py::module_::import("torch").attr("device")(dev.str());
        py::object r = f(k, shp, dv);
        return r.cast<Tensor>();
    }
    return at::empty(shape, at::TensorOptions().dtype(at::kFloat).device(dev));
}

// ---- forward / backward over the C ABI -----------------------------------------------------------
struct FwdOut {
    int64_t K = 0;
    Tensor color, invdepth, radii, geom, binning, image;
};

FwdOut forward_call(const Tensor &bg, const Tensor &means3D, const Tensor &colors, const Tensor &opacity,
                    const Tensor &scales, const Tensor &rotations, double scale_modifier, const Tensor &cov3D,
                    const Tensor &viewmatrix, const Tensor &projmatrix, double tanx, double tany, int64_t image_height,
                    int64_t image_width, const Tensor &sh, int64_t degree, const Tensor &campos, bool prefiltered,
                    bool debug, const Tensor &ri, const Tensor &pi, const Tensor &iw, const Tensor &kids, bool do_depth,
                    bool need_backward) {
    if (!means3D.defined() || means3D.dim() != 2 || means3D.size(1) != 3)
        fail("means3D must have dimensions (num_points, 3)");
    require_gpu(means3D);
    const at::Device dev = means3D.device();
    const int P = (int)means3D.size(0);
    const int H = (int)image_height, W = (int)image_width;
    const int M = present(sh) ? (int)sh.size(1) : 0;
    const Tensor means_c = dev_f32(means3D, "means3D", dev), sh_c = dev_f32(sh, "sh", dev),
                 colors_c = dev_f32(colors, "colors_precomp", dev), opac_c = dev_f32(opacity, "opacities", dev),
                 scales_c = dev_f32(scales, "scales", dev), rots_c = dev_f32(rotations, "rotations", dev),
                 cov_c = dev_f32(cov3D, "cov3D_precomp", dev), view_c = dev_f32(viewmatrix, "viewmatrix", dev),
                 proj_c = dev_f32(projmatrix, "projmatrix", dev), campos_c = dev_f32(campos, "campos", dev),
                 bg_c = dev_f32(bg, "bg", dev);
    if (P > 0 && !opac_c.defined()) fail("opacities must be provided");
    const Cut cut = cut_args(ri, pi, iw, kids, dev);
    const auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
    FwdOut o;
    o.color = at::empty({3, H, W}, f32);
    // written for every pixel when do_depth; zeros otherwise (callers ignore it)
    o.invdepth = do_depth ? at::empty({1, H, W}, f32) : at::zeros({1, H, W}, f32);
    o.radii = at::empty({cut.n > 0 ? cut.n : P}, at::TensorOptions().dtype(at::kInt).device(dev));
    Buffers b{at::TensorOptions().dtype(at::kByte).device(dev)};
    int rc;
    {
        c10::DeviceGuard guard(dev);
        void *s = stream_of(dev);
        NoGil nogil;
        rc = abi().forward_ex(
            resize_geom, resize_binning, resize_image, &b, P, (int)degree, M, fp(bg_c), W, H, fp(means_c), fp(sh_c),
            fp(colors_c), fp(opac_c), fp(scales_c), (float)scale_modifier, fp(rots_c), fp(cov_c), fp(view_c),
            fp(proj_c), fp(campos_c), (float)tanx, (float)tany, prefiltered ? 1 : 0, wp(o.color),
            do_depth ? wp(o.invdepth) : nullptr, ptr<int>(o.radii), ptr<const int>(cut.ri), ptr<const int>(cut.pi),
            fp(cut.w), ptr<const int>(cut.kids), cut.n, debug ? 1 : 0, s, &o.K, need_backward ? 0u : GSR_FWD_NO_BACKWARD);
    }
    check_call(rc, "rasterize_gaussians", b);
    o.geom = u8_or_empty(b.geom, dev);
    o.binning = u8_or_empty(b.binning, dev);
    o.image = u8_or_empty(b.image, dev);
    return o;
}

struct BwdOut {
    Tensor dmeans2D, dcolors, dopacity, dmeans3D, dcov3D, dsh, dscales, drots;
};

BwdOut backward_call(const Tensor &bg, const Tensor &means3D, const Tensor &radii, const Tensor &colors,
                     const Tensor &scales, const Tensor &rotations, double scale_modifier, const Tensor &cov3D,
                     const Tensor &viewmatrix, const Tensor &projmatrix, double tanx, double tany,
                     const Tensor &dL_dcolor, const Tensor &dL_dinvdepth, const Tensor &sh, int64_t degree,
                     const Tensor &campos, const Tensor &geom, int64_t R, const Tensor &binning, const Tensor &image,
                     const Tensor &ri, const Tensor &pi, const Tensor &iw, const Tensor &kids, bool debug,
                     bool validated) {
    require_gpu(means3D);
    const at::Device dev = means3D.device();
    const int P = (int)means3D.size(0);
    const int H = (int)dL_dcolor.size(1), W = (int)dL_dcolor.size(2);
    const int M = present(sh) ? (int)sh.size(1) : 0;
    Tensor means_c, sh_c, colors_c, scales_c, rots_c, cov_c, view_c, proj_c, campos_c, bg_c;
    if (validated) {  // the autograd Function's own forward checked these tensors
        means_c = saved(means3D), sh_c = saved(sh), colors_c = saved(colors), scales_c = saved(scales),
        rots_c = saved(rotations), cov_c = saved(cov3D), view_c = saved(viewmatrix), proj_c = saved(projmatrix),
        campos_c = saved(campos), bg_c = saved(bg);
    } else {
        means_c = dev_f32(means3D, "means3D", dev), sh_c = dev_f32(sh, "sh", dev),
        colors_c = dev_f32(colors, "colors_precomp", dev), scales_c = dev_f32(scales, "scales", dev),
        rots_c = dev_f32(rotations, "rotations", dev), cov_c = dev_f32(cov3D, "cov3D_precomp", dev),
        view_c = dev_f32(viewmatrix, "viewmatrix", dev), proj_c = dev_f32(projmatrix, "projmatrix", dev),
        campos_c = dev_f32(campos, "campos", dev), bg_c = dev_f32(bg, "bg", dev);
    }
    const Tensor dpix = dev_f32(dL_dcolor, "dL_dout_color", dev);
    const Tensor dinv = dL_dinvdepth.defined() ? dev_f32(dL_dinvdepth, "dL_dout_invdepth", dev) : Tensor();
    const Tensor radii_c = radii.contiguous();
    const Cut cut = cut_args(ri, pi, iw, kids, dev);

    const auto f32 = at::TensorOptions().dtype(at::kFloat).device(dev);
    // gradients of inputs that were not given are identically zero: zero-stride views (upstream's
    // shapes, no memory traffic), not computed by the kernels
    const auto z = [&](std::initializer_list<int64_t> shape) { return zero_of(dev).expand(shape); };
    BwdOut g;
    g.dmeans2D = at::empty({P, 3}, f32);
    g.dopacity = at::empty({P, 1}, f32);
    g.dmeans3D = leaf_grad(means3D, {P, 3}, dev);
    g.dcolors = sh_c.defined() ? z({P, 3}) : at::empty({P, 3}, f32);
    g.dcov3D = cov_c.defined() ? at::empty({P, 6}, f32) : z({P, 6});
    g.dsh = sh_c.defined() ? leaf_grad(sh, {P, M, 3}, dev) : at::zeros({P, 0, 3}, f32);
    if (!cov_c.defined()) {
        g.dscales = at::empty({P, 3}, f32);
        g.drots = at::empty({P, 4}, f32);
    } else {
        g.dscales = z({P, 3});
        g.drots = z({P, 4});
    }
    Buffers b{at::TensorOptions().dtype(at::kByte).device(dev)};
    int rc;
    {
        c10::DeviceGuard guard(dev);
        void *s = stream_of(dev);
        NoGil nogil;
        rc = abi().backward(
            resize_scratch, &b, P, (int)degree, M, R, fp(bg_c), W, H, fp(means_c), fp(sh_c), fp(colors_c),
            fp(scales_c), (float)scale_modifier, fp(rots_c), fp(cov_c), fp(view_c), fp(proj_c), fp(campos_c),
            (float)tanx, (float)tany, ptr<const int>(radii_c), geom.data_ptr(), binning.data_ptr(), image.data_ptr(),
            fp(dpix), fp(dinv), wp(g.dmeans2D), sh_c.defined() ? nullptr : wp(g.dcolors), wp(g.dopacity),
            wp(g.dmeans3D), cov_c.defined() ? wp(g.dcov3D) : nullptr, sh_c.defined() ? wp(g.dsh) : nullptr,
            cov_c.defined() ? nullptr : wp(g.dscales), cov_c.defined() ? nullptr : wp(g.drots),
            ptr<const int>(cut.ri), ptr<const int>(cut.pi), fp(cut.w), ptr<const int>(cut.kids), cut.n, debug ? 1 : 0,
            s);
    }
    check_call(rc, "rasterize_gaussians_backward", b);
    return g;
}

// Optional tensor argument from Python: None -> undefined
Tensor opt(const std::optional<Tensor> &t) { return t.has_value() ? *t : Tensor(); }

// ---- the autograd Function ------------------------------------------------------------------------
// GaussianRasterizationSettings, read once per call (getattr: the hierarchy fields may be missing
// from a caller's own settings type, as in _RasterizeGaussians.forward)
struct Settings {
    int64_t H = 0, W = 0, degree = 0;
    double tanx = 0, tany = 0, scale_modifier = 1;
    bool prefiltered = false, debug = false, do_depth = true;
    Tensor bg, view, proj, campos, ri, pi, iw, kids;
};

Tensor tensor_attr(const py::handle &rs, const char *name) {
    if (!py::hasattr(rs, name)) return Tensor();
    py::object v = rs.attr(name);
    if (v.is_none()) return Tensor();
    return v.cast<Tensor>();
}

Settings read_settings(const py::handle &rs) {
    Settings s;
    s.H = rs.attr("image_height").cast<int64_t>();
    s.W = rs.attr("image_width").cast<int64_t>();
    s.tanx = rs.attr("tanfovx").cast<double>();
    s.tany = rs.attr("tanfovy").cast<double>();
    s.bg = rs.attr("bg").cast<Tensor>();
    s.scale_modifier = rs.attr("scale_modifier").cast<double>();
    s.view = rs.attr("viewmatrix").cast<Tensor>();
    s.proj = rs.attr("projmatrix").cast<Tensor>();
    s.degree = rs.attr("sh_degree").cast<int64_t>();
    s.campos = rs.attr("campos").cast<Tensor>();
    s.prefiltered = py::bool_(rs.attr("prefiltered"));
    s.debug = py::bool_(rs.attr("debug"));
    s.do_depth = py::hasattr(rs, "do_depth") ? bool(py::bool_(rs.attr("do_depth"))) : true;
    s.ri = tensor_attr(rs, "render_indices");
    s.pi = tensor_attr(rs, "parent_indices");
    s.iw = tensor_attr(rs, "interpolation_weights");
    s.kids = tensor_attr(rs, "num_node_kids");
    return s;
}

struct RasterizeFn : public torch::autograd::Function<RasterizeFn> {
    static variable_list forward(AutogradContext *ctx, const Tensor &means3D, const Tensor &means2D, const Tensor &sh,
                                 const Tensor &colors, const Tensor &opacities, const Tensor &scales,
                                 const Tensor &rotations, const Tensor &cov3D, const Settings &rs, bool need_backward) {
        (void)means2D;  // receives the screen-space gradient only
        FwdOut o = forward_call(rs.bg, means3D, colors, opacities, scales, rotations, rs.scale_modifier, cov3D, rs.view,
                                rs.proj, rs.tanx, rs.tany, rs.H, rs.W, sh, rs.degree, rs.campos, rs.prefiltered,
                                rs.debug, rs.ri, rs.pi, rs.iw, rs.kids, rs.do_depth, need_backward);
        // an output no loss uses (the inverse depth, in most training steps) arrives undefined, not
        // as a materialised zero image: the backward then skips its depth term
        ctx->set_materialize_grads(false);
        ctx->saved_data["K"] = o.K;
        ctx->saved_data["do_depth"] = rs.do_depth;
        ctx->saved_data["H"] = rs.H;
        ctx->saved_data["W"] = rs.W;
        ctx->saved_data["degree"] = rs.degree;
        ctx->saved_data["tanx"] = rs.tanx;
        ctx->saved_data["tany"] = rs.tany;
        ctx->saved_data["scale_modifier"] = rs.scale_modifier;
        ctx->saved_data["debug"] = rs.debug;
        ctx->save_for_backward({colors, means3D, scales, rotations, cov3D, o.radii, sh, o.geom, o.binning, o.image,
                                rs.bg, rs.view, rs.proj, rs.campos, rs.ri, rs.pi, rs.iw, rs.kids});
        ctx->mark_non_differentiable({o.radii});
        return {o.color, o.radii, o.invdepth};
    }

    static variable_list backward(AutogradContext *ctx, variable_list grad_out) {
        const auto sv = ctx->get_saved_variables();
        const Tensor &colors = sv[0], &means3D = sv[1], &scales = sv[2], &rotations = sv[3], &cov3D = sv[4],
                     &radii = sv[5], &sh = sv[6], &geom = sv[7], &binning = sv[8], &image = sv[9], &bg = sv[10],
                     &view = sv[11], &proj = sv[12], &campos = sv[13], &ri = sv[14], &pi = sv[15], &iw = sv[16],
                     &kids = sv[17];
        const int64_t H = ctx->saved_data["H"].toInt(), W = ctx->saved_data["W"].toInt();
        Tensor gcol = grad_out[0];
        if (!gcol.defined())
            gcol = at::zeros({3, H, W}, at::TensorOptions().dtype(at::kFloat).device(means3D.device()));
        const Tensor ginv = ctx->saved_data["do_depth"].toBool() && grad_out[2].defined() ? grad_out[2].contiguous()
                                                                                          : Tensor();
        BwdOut g = backward_call(bg, means3D, radii, colors, scales, rotations, ctx->saved_data["scale_modifier"].toDouble(),
                                 cov3D, view, proj, ctx->saved_data["tanx"].toDouble(), ctx->saved_data["tany"].toDouble(),
                                 gcol.contiguous(), ginv, sh, ctx->saved_data["degree"].toInt(), campos, geom,
                                 ctx->saved_data["K"].toInt(), binning, image, ri, pi, iw, kids,
                                 ctx->saved_data["debug"].toBool(), /*validated=*/true);
        const auto keep = [](const Tensor &gr, const Tensor &inp) { return present(inp) ? gr : Tensor(); };
        // (means3D, means2D, sh, colors_precomp, opacities, scales, rotations, cov3D_precomp, settings, need_backward)
        return {g.dmeans3D, g.dmeans2D, keep(g.dsh, sh), keep(g.dcolors, colors), g.dopacity, keep(g.dscales, scales),
                keep(g.drots, rotations), keep(g.dcov3D, cov3D), Tensor(), Tensor()};
    }
};

bool any_requires_grad(std::initializer_list<const Tensor *> ts) {
    for (const Tensor *t : ts)
        if (t->defined() && t->requires_grad()) return true;
    return false;
}

py::tuple rasterize(const Tensor &means3D, const Tensor &means2D, const std::optional<Tensor> &sh,
                    const std::optional<Tensor> &colors, const Tensor &opacities, const std::optional<Tensor> &scales,
                    const std::optional<Tensor> &rotations, const std::optional<Tensor> &cov3D, py::handle rs_obj) {
    const Settings rs = read_settings(rs_obj);
    const Tensor sh_t = opt(sh), col_t = opt(colors), sc_t = opt(scales), rot_t = opt(rotations), cov_t = opt(cov3D);
    // a frame autograd will not record (torch.no_grad evaluation, or no input that requires grad)
    // can never reach the backward: it skips the backward's accumulator clear
    const bool need_backward =
        at::GradMode::is_enabled() &&
        any_requires_grad({&means3D, &means2D, &sh_t, &col_t, &opacities, &sc_t, &rot_t, &cov_t});
    variable_list out = RasterizeFn::apply(means3D, means2D, sh_t, col_t, opacities, sc_t, rot_t, cov_t, rs, need_backward);
    return py::make_tuple(out[0], out[1], out[2]);
}

py::tuple rasterize_gaussians(const std::optional<Tensor> &bg, const Tensor &means3D, const std::optional<Tensor> &colors,
                              const std::optional<Tensor> &opacity, const std::optional<Tensor> &scales,
                              const std::optional<Tensor> &rotations, double scale_modifier,
                              const std::optional<Tensor> &cov3D, const std::optional<Tensor> &viewmatrix,
                              const std::optional<Tensor> &projmatrix, double tanx, double tany, int64_t H, int64_t W,
                              const std::optional<Tensor> &sh, int64_t degree, const std::optional<Tensor> &campos,
                              bool prefiltered, bool debug, const std::optional<Tensor> &ri,
                              const std::optional<Tensor> &pi, const std::optional<Tensor> &iw,
                              const std::optional<Tensor> &kids, bool do_depth, bool need_backward) {
    FwdOut o = forward_call(opt(bg), means3D, opt(colors), opt(opacity), opt(scales), opt(rotations), scale_modifier,
                            opt(cov3D), opt(viewmatrix), opt(projmatrix), tanx, tany, H, W, opt(sh), degree, opt(campos),
                            prefiltered, debug, opt(ri), opt(pi), opt(iw), opt(kids), do_depth, need_backward);
    return py::make_tuple(o.K, o.color, o.invdepth, o.radii, o.geom, o.binning, o.image);
}

py::tuple rasterize_gaussians_backward(
    const std::optional<Tensor> &bg, const Tensor &means3D, const Tensor &radii, const std::optional<Tensor> &colors,
    const std::optional<Tensor> &scales, const std::optional<Tensor> &rotations, double scale_modifier,
    const std::optional<Tensor> &cov3D, const std::optional<Tensor> &viewmatrix, const std::optional<Tensor> &projmatrix,
    double tanx, double tany, const Tensor &dL_dcolor, const std::optional<Tensor> &dL_dinvdepth,
    const std::optional<Tensor> &sh, int64_t degree, const std::optional<Tensor> &campos, const Tensor &geom, int64_t R,
    const Tensor &binning, const Tensor &image, const std::optional<Tensor> &ri, const std::optional<Tensor> &pi,
    const std::optional<Tensor> &iw, const std::optional<Tensor> &kids, bool debug, bool validated) {
    BwdOut g = backward_call(opt(bg), means3D, radii, opt(colors), opt(scales), opt(rotations), scale_modifier,
                             opt(cov3D), opt(viewmatrix), opt(projmatrix), tanx, tany, dL_dcolor, opt(dL_dinvdepth),
                             opt(sh), degree, opt(campos), geom, R, binning, image, opt(ri), opt(pi), opt(iw), opt(kids),
                             debug, validated);
    return py::make_tuple(g.dmeans2D, g.dcolors, g.dopacity, g.dmeans3D, g.dcov3D, g.dsh, g.dscales, g.drots);
}

Tensor mark_visible(const Tensor &means3D, const Tensor &viewmatrix, const Tensor &projmatrix) {
    require_gpu(means3D);
    const at::Device dev = means3D.device();
    const int P = (int)means3D.size(0);
    Tensor present_ = at::empty({P}, at::TensorOptions().dtype(at::kByte).device(dev));
    const Tensor m = dev_f32(means3D, "means3D", dev), v = dev_f32(viewmatrix, "viewmatrix", dev),
                 p = dev_f32(projmatrix, "projmatrix", dev);
    int rc;
    {
        c10::DeviceGuard guard(dev);
        rc = abi().mark_visible(P, fp(m), fp(v), fp(p), ptr<uint8_t>(present_), stream_of(dev));
    }
    check(rc, "mark_visible");
    return present_.to(at::kBool);
}

void set_grad_provider(py::object f) {  // called with the GIL held
    PyObject *old = g_provider;
    g_provider = f.is_none() ? nullptr : f.inc_ref().ptr();
    g_provider_set.store(g_provider != nullptr, std::memory_order_release);
    Py_XDECREF(old);
}

}  // namespace

PYBIND11_MODULE(_gsr_host, m) {
    m.doc() = "MI355X rasterizer host path (C++ over libgsr_hip.so's C ABI)";
    m.def("bind", &bind, py::arg("library_path"));
    m.def("rasterize", &rasterize, py::arg("means3D"), py::arg("means2D"), py::arg("sh"), py::arg("colors_precomp"),
          py::arg("opacities"), py::arg("scales"), py::arg("rotations"), py::arg("cov3D_precomp"),
          py::arg("raster_settings"));
    m.def("rasterize_gaussians", &rasterize_gaussians, py::arg("background"), py::arg("means3D"), py::arg("colors"),
          py::arg("opacity"), py::arg("scales"), py::arg("rotations"), py::arg("scale_modifier"),
          py::arg("cov3D_precomp"), py::arg("viewmatrix"), py::arg("projmatrix"), py::arg("tan_fovx"),
          py::arg("tan_fovy"), py::arg("image_height"), py::arg("image_width"), py::arg("sh"), py::arg("degree"),
          py::arg("campos"), py::arg("prefiltered"), py::arg("debug"), py::arg("render_indices") = py::none(),
          py::arg("parent_indices") = py::none(), py::arg("interpolation_weights") = py::none(),
          py::arg("num_node_kids") = py::none(), py::arg("do_depth") = true, py::arg("need_backward") = true);
    m.def("rasterize_gaussians_backward", &rasterize_gaussians_backward, py::arg("background"), py::arg("means3D"),
          py::arg("radii"), py::arg("colors"), py::arg("scales"), py::arg("rotations"), py::arg("scale_modifier"),
          py::arg("cov3D_precomp"), py::arg("viewmatrix"), py::arg("projmatrix"), py::arg("tan_fovx"),
          py::arg("tan_fovy"), py::arg("dL_dout_color"), py::arg("dL_dout_invdepth"), py::arg("sh"), py::arg("degree"),
          py::arg("campos"), py::arg("geomBuffer"), py::arg("R"), py::arg("binningBuffer"), py::arg("imageBuffer"),
          py::arg("render_indices") = py::none(), py::arg("parent_indices") = py::none(),
          py::arg("interpolation_weights") = py::none(), py::arg("num_node_kids") = py::none(),
          py::arg("debug") = false, py::arg("validated") = false);
    m.def("mark_visible", &mark_visible, py::arg("means3D"), py::arg("viewmatrix"), py::arg("projmatrix"));
    m.def("set_grad_provider", &set_grad_provider, py::arg("provider"));
}
