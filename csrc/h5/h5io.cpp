// Minimal native HDF5 writer/reader for Keras-layout checkpoints.
//
// Reference: every script ends with model.save('ImageNet-<name>-reuse.h5')
// (imagenet-resnet50.py:69-72), i.e. the Keras HDF5 full-model format; pretrained variants
// load Keras' ResNet50 `..._notop.h5` weights (imagenet-pretrained-resnet50.py:56).  This
// module (`_pddl_h5`, linked against libhdf5 1.10) exposes exactly what the Python layer
// (utils/checkpoint.py) needs to produce / consume that layout:
//   write(path, datasets, attrs)       datasets: [(name, ndarray float32|int64)], intermediate
//                                      groups created; attrs: [(object, name, str | [str])]
//                                      (str -> variable-length UTF-8 scalar like h5py; [str] ->
//                                      fixed-length NULL-padded byte strings like Keras)
//   read_dataset(path, name) -> ndarray
//   read_attr(path, object, name) -> str | [str]
//   list_datasets(path) -> [name]
#include <hdf5.h>
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include <stdexcept>
#include <string>
#include <vector>

namespace py = pybind11;

namespace {

void chk(herr_t r, const std::string& what) {
  if (r < 0) throw std::runtime_error("pddl h5: " + what);
}
hid_t chkid(hid_t id, const std::string& what) {
  if (id < 0) throw std::runtime_error("pddl h5: " + what);
  return id;
}

struct Handle {
  hid_t id;
  herr_t (*closer)(hid_t);
  Handle(hid_t i, herr_t (*c)(hid_t)) : id(i), closer(c) {}
  ~Handle() {
    if (id >= 0) closer(id);
  }
  operator hid_t() const { return id; }
};

void ensure_group(hid_t file, const std::string& path) {
  if (path.empty() || path == "/") return;
  std::string cur;
  size_t pos = 0;
  while (pos <= path.size()) {
    size_t nx = path.find('/', pos);
    if (nx == std::string::npos) nx = path.size();
    const std::string part = path.substr(pos, nx - pos);
    if (!part.empty()) {
      cur += "/" + part;
      if (H5Lexists(file, cur.c_str(), H5P_DEFAULT) <= 0) {
        Handle g(chkid(H5Gcreate2(file, cur.c_str(), H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT), "create group " + cur),
                 H5Gclose);
      }
    }
    pos = nx + 1;
  }
}

void write_dataset(hid_t file, const std::string& name, py::array arr) {
  const size_t slash = name.rfind('/');
  if (slash != std::string::npos) ensure_group(file, name.substr(0, slash));
  std::vector<hsize_t> dims(arr.ndim());
  for (int i = 0; i < arr.ndim(); ++i) dims[i] = (hsize_t)arr.shape(i);
  Handle space(arr.ndim() == 0 ? H5Screate(H5S_SCALAR) : H5Screate_simple(arr.ndim(), dims.data(), nullptr),
               H5Sclose);
  hid_t mem_t, file_t;
  if (py::isinstance<py::array_t<float>>(arr)) {
    mem_t = H5T_NATIVE_FLOAT;
    file_t = H5T_IEEE_F32LE;
  } else if (py::isinstance<py::array_t<int64_t>>(arr)) {
    mem_t = H5T_NATIVE_INT64;
    file_t = H5T_STD_I64LE;
  } else {
    throw std::runtime_error("pddl h5: datasets must be float32 or int64 (" + name + ")");
  }
  auto c = py::array::ensure(arr, py::array::c_style);
  Handle ds(chkid(H5Dcreate2(file, name.c_str(), file_t, space, H5P_DEFAULT, H5P_DEFAULT, H5P_DEFAULT),
                  "create dataset " + name),
            H5Dclose);
  chk(H5Dwrite(ds, mem_t, H5S_ALL, H5S_ALL, H5P_DEFAULT, c.data()), "write dataset " + name);
}

void write_attr(hid_t file, const std::string& obj, const std::string& name, py::handle value) {
  ensure_group(file, obj);
  Handle o(chkid(H5Oopen(file, obj.empty() ? "/" : obj.c_str(), H5P_DEFAULT), "open object " + obj), H5Oclose);
  if (H5Aexists(o, name.c_str()) > 0) chk(H5Adelete(o, name.c_str()), "delete attr");
  if (py::isinstance<py::str>(value) || py::isinstance<py::bytes>(value)) {
    const std::string v = py::cast<std::string>(value);
    Handle t(H5Tcopy(H5T_C_S1), H5Tclose);
    chk(H5Tset_size(t, H5T_VARIABLE), "tset");
    chk(H5Tset_cset(t, H5T_CSET_UTF8), "cset");
    Handle sp(H5Screate(H5S_SCALAR), H5Sclose);
    Handle a(chkid(H5Acreate2(o, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), "create attr " + name), H5Aclose);
    const char* p = v.c_str();
    chk(H5Awrite(a, t, &p), "write attr " + name);
    return;
  }
  std::vector<std::string> vs = py::cast<std::vector<std::string>>(value);
  size_t mx = 1;
  for (auto& s : vs) mx = std::max(mx, s.size());
  std::vector<char> buf(vs.size() * mx, 0);
  for (size_t i = 0; i < vs.size(); ++i) memcpy(buf.data() + i * mx, vs[i].data(), vs[i].size());
  Handle t(H5Tcopy(H5T_C_S1), H5Tclose);
  chk(H5Tset_size(t, mx), "tset");
  chk(H5Tset_strpad(t, H5T_STR_NULLPAD), "strpad");
  hsize_t n = vs.size();
  Handle sp(H5Screate_simple(1, &n, nullptr), H5Sclose);
  Handle a(chkid(H5Acreate2(o, name.c_str(), t, sp, H5P_DEFAULT, H5P_DEFAULT), "create attr " + name), H5Aclose);
  if (n) chk(H5Awrite(a, t, buf.data()), "write attr " + name);
}

void h5_write(const std::string& path, std::vector<std::pair<std::string, py::array>> datasets,
           std::vector<std::tuple<std::string, std::string, py::object>> attrs) {
  Handle f(chkid(H5Fcreate(path.c_str(), H5F_ACC_TRUNC, H5P_DEFAULT, H5P_DEFAULT), "create " + path), H5Fclose);
  for (auto& kv : datasets) write_dataset(f, kv.first, kv.second);
  for (auto& a : attrs) write_attr(f, std::get<0>(a), std::get<1>(a), std::get<2>(a));
}

py::array read_dataset(const std::string& path, const std::string& name) {
  Handle f(chkid(H5Fopen(path.c_str(), H5F_ACC_RDONLY, H5P_DEFAULT), "open " + path), H5Fclose);
  Handle ds(chkid(H5Dopen2(f, name.c_str(), H5P_DEFAULT), "open dataset " + name), H5Dclose);
  Handle sp(H5Dget_space(ds), H5Sclose);
  const int nd = H5Sget_simple_extent_ndims(sp);
  std::vector<hsize_t> dims(nd > 0 ? nd : 0);
  if (nd > 0) H5Sget_simple_extent_dims(sp, dims.data(), nullptr);
  std::vector<py::ssize_t> shape(dims.begin(), dims.end());
  Handle t(H5Dget_type(ds), H5Tclose);
  if (H5Tget_class(t) == H5T_INTEGER) {
    py::array_t<int64_t> out(shape);
    chk(H5Dread(ds, H5T_NATIVE_INT64, H5S_ALL, H5S_ALL, H5P_DEFAULT, out.mutable_data()), "read " + name);
    return out;
  }
  py::array_t<float> out(shape);
  chk(H5Dread(ds, H5T_NATIVE_FLOAT, H5S_ALL, H5S_ALL, H5P_DEFAULT, out.mutable_data()), "read " + name);
  return out;
}

py::object read_attr(const std::string& path, const std::string& obj, const std::string& name) {
  Handle f(chkid(H5Fopen(path.c_str(), H5F_ACC_RDONLY, H5P_DEFAULT), "open " + path), H5Fclose);
  if (H5Aexists_by_name(f, obj.empty() ? "/" : obj.c_str(), name.c_str(), H5P_DEFAULT) <= 0) return py::none();
  Handle a(chkid(H5Aopen_by_name(f, obj.empty() ? "/" : obj.c_str(), name.c_str(), H5P_DEFAULT, H5P_DEFAULT),
                 "open attr " + name),
           H5Aclose);
  Handle t(H5Aget_type(a), H5Tclose);
  Handle sp(H5Aget_space(a), H5Sclose);
  const hssize_t n = H5Sget_simple_extent_npoints(sp);
  const bool scalar = H5Sget_simple_extent_type(sp) == H5S_SCALAR;
  if (H5Tget_class(t) != H5T_STRING) {
    double v = 0;
    chk(H5Aread(a, H5T_NATIVE_DOUBLE, &v), "read attr");
    return py::float_(v);
  }
  std::vector<std::string> vals;
  if (H5Tis_variable_str(t) > 0) {
    std::vector<char*> ptrs(n);
    Handle mt(H5Tcopy(H5T_C_S1), H5Tclose);
    H5Tset_size(mt, H5T_VARIABLE);
    H5Tset_cset(mt, H5Tget_cset(t));
    chk(H5Aread(a, mt, ptrs.data()), "read vlen attr");
    for (auto p : ptrs) vals.emplace_back(p ? p : "");
    H5Dvlen_reclaim(mt, sp, H5P_DEFAULT, ptrs.data());
  } else {
    const size_t sz = H5Tget_size(t);
    std::vector<char> buf(n * sz + 1, 0);
    chk(H5Aread(a, t, buf.data()), "read attr");
    for (hssize_t i = 0; i < n; ++i) vals.emplace_back(strnlen(buf.data() + i * sz, sz) ? std::string(buf.data() + i * sz, strnlen(buf.data() + i * sz, sz)) : "");
  }
  if (scalar) return py::str(vals.empty() ? "" : vals[0]);
  return py::cast(vals);
}

herr_t visit_cb(hid_t, const char* name, const H5O_info_t* info, void* data) {
  if (info->type == H5O_TYPE_DATASET) static_cast<std::vector<std::string>*>(data)->push_back(name);
  return 0;
}

std::vector<std::string> list_datasets(const std::string& path) {
  Handle f(chkid(H5Fopen(path.c_str(), H5F_ACC_RDONLY, H5P_DEFAULT), "open " + path), H5Fclose);
  std::vector<std::string> out;
  chk(H5Ovisit(f, H5_INDEX_NAME, H5_ITER_NATIVE, visit_cb, &out), "visit");
  return out;
}

}  // namespace

PYBIND11_MODULE(_pddl_h5, m) {
  m.doc() = "pddl native HDF5 I/O for Keras-layout checkpoints";
  m.def("write", &h5_write);
  m.def("read_dataset", &read_dataset);
  m.def("read_attr", &read_attr);
  m.def("list_datasets", &list_datasets);
  m.attr("HDF5_VERSION") = H5_VERS_INFO;
}
