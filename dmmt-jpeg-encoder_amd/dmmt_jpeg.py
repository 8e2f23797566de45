"""Python host mirror of the reference encoder API over the gfx950 C ABI.

The reference (SilverlightningY/dmmt-jpeg-encoder) is a Rust crate whose public
seam is ``JpegImageWriter::write_image`` (src/image/writer/jpeg.rs:64-75),
reached from ``convert_ppm_to_jpeg`` (src/lib.rs:59-77).  This module mirrors
those names, their argument meaning and their error behaviour, and calls
``lib/libdmmt_jpeg.so`` (include/dmmt_jpeg.h) through ctypes.  All compute runs
on the GPU; when the library or a gfx950 device is missing this module raises --
it never falls back to a CPU path.

One HIP runtime per process: torch wheels bundle their own libamdhip64.so.7.
If torch is importable it is imported *before* the library is loaded so that
both bind to the same runtime (loading ours first and torch afterwards would map
two runtimes into one process).
"""
from __future__ import annotations

import ctypes
import enum
import io
import os
import subprocess
from dataclasses import dataclass

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
# DMMT_LIB_PATH selects another build of the same library (e.g. the
# `make TRACE=1` development build in lib_trace/)
LIB_PATH = os.environ.get("DMMT_LIB_PATH") or os.path.join(_HERE, "lib", "libdmmt_jpeg.so")
CLI_PATH = os.path.join(_HERE, "bin", "dmmt-jpeg-encoder")

try:  # see module docstring: bind the library to torch's HIP runtime if torch is present
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the product
    torch = None

_lib = None

# ---------------------------------------------------------------- errors


class Error(Exception):
    """error::Error (src/error.rs:3-22) plus the states where the reference panics."""

    PPM_CODES = (-1, -2, -3)  # the variants with a payload (error.rs:4-7)

    def __init__(self, code: int, context: str = ""):
        self.code = code
        self.name = lib().dmmt_error_name(code).decode() if _lib is not None else str(code)
        msg = lib().dmmt_strerror(code).decode() if _lib is not None else str(code)
        # the variant's payload (read right after the failing call, same thread):
        # IncompletePixelParsed(n) -> n; the token index of the two token errors
        self.detail = lib().dmmt_last_error_detail() if _lib is not None and code in self.PPM_CODES else None
        self.n = self.detail if code == -3 else None
        if self.detail is not None:
            msg = lib().dmmt_last_error_message().decode()
        super().__init__(f"{self.name}: {msg}" + (f" ({context})" if context else ""))


class LibraryMissing(RuntimeError):
    pass


def build() -> str:
    """Compile the HIP library and CLI in-tree (hipcc --offload-arch=gfx950)."""
    subprocess.run(["make", "-s", "-C", _HERE, "-j8"], check=True)
    return LIB_PATH


def lib():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise LibraryMissing(f"{LIB_PATH} is not built; run build() or `make -C {_HERE}` -- there is no CPU fallback")
    L = ctypes.CDLL(LIB_PATH)
    vp, sz, i32, u16 = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_uint16
    P = ctypes.POINTER
    L.dmmt_ctx_create.argtypes = [ctypes.c_int, P(vp)]
    L.dmmt_ctx_destroy.argtypes = [vp]
    L.dmmt_ctx_destroy.restype = None
    L.dmmt_device_count.argtypes = [P(ctypes.c_int)]
    L.dmmt_ctx_synchronize.argtypes = [vp]
    L.dmmt_jpeg_encode.argtypes = [vp, P(DmmtImage), P(DmmtOptions), P(vp), P(sz)]
    L.dmmt_jpeg_encode_batch.argtypes = [vp, P(DmmtImage), ctypes.c_int, P(DmmtOptions), P(vp), P(sz)]
    L.dmmt_encode_device.argtypes = [vp, P(DmmtDeviceFrames), P(DmmtOptions), vp]
    L.dmmt_ctx_set_lanes.argtypes = [vp, ctypes.c_int]
    L.dmmt_max_jpeg_bytes.argtypes = [u16, u16, i32]
    L.dmmt_max_jpeg_bytes.restype = sz
    L.dmmt_forward_blocks.argtypes = [vp, P(DmmtImage), P(DmmtOptions), vp, sz, P(sz)]
    L.dmmt_encode_coefficients.argtypes = [vp, vp, sz, u16, u16, P(DmmtOptions), P(vp), P(sz)]
    L.dmmt_dct_transform.argtypes = [vp, vp, sz]
    L.dmmt_quantization_preset.argtypes = [i32, vp, vp]
    L.dmmt_quality_tables.argtypes = [i32, vp, vp]
    L.dmmt_default_options.argtypes = [P(DmmtOptions)]
    L.dmmt_default_options.restype = None
    L.dmmt_read_ppm.argtypes = [ctypes.c_char_p, P(DmmtImage)]
    L.dmmt_parse_ppm.argtypes = [vp, sz, P(DmmtImage)]
    L.dmmt_convert_ppm_to_jpeg.argtypes = [vp, ctypes.c_char_p, ctypes.c_char_p, P(DmmtOptions)]
    L.dmmt_parse_ppm_header.argtypes = [vp, sz, P(DmmtPpmHeader)]
    L.dmmt_decode_ppm_device.argtypes = [vp, vp, sz, P(DmmtPpmHeader), vp, vp]
    L.dmmt_convert_ppm_device_batch.argtypes = [vp, P(DmmtPpmFile), i32, P(DmmtOptions), P(i32)]
    L.dmmt_ctx_batch_redone.argtypes = [vp]
    L.dmmt_ctx_check_device.argtypes = [vp, P(i32)]
    L.dmmt_free.argtypes = [vp]
    L.dmmt_free.restype = None
    L.dmmt_strerror.argtypes = [ctypes.c_int]
    L.dmmt_strerror.restype = ctypes.c_char_p
    L.dmmt_error_name.argtypes = [ctypes.c_int]
    L.dmmt_error_name.restype = ctypes.c_char_p
    L.dmmt_ctx_set_profiling.argtypes = [vp, ctypes.c_int]
    L.dmmt_ctx_profile.argtypes = [vp, P(ctypes.c_double), P(i32), ctypes.c_int]
    L.dmmt_num_stages.argtypes = []
    L.dmmt_stage_name.argtypes = [ctypes.c_int]
    L.dmmt_stage_name.restype = ctypes.c_char_p
    L.dmmt_device_malloc.argtypes = [vp, sz, P(vp)]
    L.dmmt_device_free.argtypes = [vp, vp]
    L.dmmt_memcpy_h2d.argtypes = [vp, vp, vp, sz]
    L.dmmt_memcpy_d2h.argtypes = [vp, vp, vp, sz]
    L.dmmt_fill_synthetic.argtypes = [vp, vp, u16, u16, i32, i32, ctypes.c_uint32]
    L.dmmt_fill_synthetic_rows.argtypes = [vp, vp, u16, u16, i32, i32, i32, ctypes.c_uint32]
    H = ctypes.c_uint64 * STRIPE_HIST_WORDS
    L.dmmt_stripe_analyze.argtypes = [vp, P(DmmtStripe), P(DmmtOptions), H]
    L.dmmt_stripe_encode.argtypes = [vp, H, vp, sz, P(ctypes.c_uint64)]
    L.dmmt_stripe_max_bytes.argtypes = [P(DmmtStripe), P(DmmtOptions)]
    L.dmmt_stripe_max_bytes.restype = sz
    I3 = ctypes.c_int16 * 3
    L.dmmt_stripe_dc_edges.argtypes = [vp, I3, I3]
    L.dmmt_stripe_fix_dc_hist.argtypes = [H, I3, I3]
    L.dmmt_stripe_fix_dc_hist.restype = None
    L.dmmt_stripe_measure.argtypes = [vp, H, I3, vp, sz, P(ctypes.c_uint64), P(ctypes.c_uint32)]
    L.dmmt_stripe_write.argtypes = [vp, ctypes.c_uint64, ctypes.c_uint32, ctypes.c_uint32, P(ctypes.c_uint64)]
    L.dmmt_ctx_create_multi.argtypes = [P(ctypes.c_int), ctypes.c_int, P(vp)]
    L.dmmt_ctx_num_devices.argtypes = [vp]
    L.dmmt_ctx_member.argtypes = [vp, ctypes.c_int]
    L.dmmt_ctx_member.restype = vp
    L.dmmt_jpeg_encode_striped.argtypes = [vp, P(DmmtImage), P(DmmtOptions), ctypes.c_int, P(vp), P(sz)]
    L.dmmt_encode_device_multi.argtypes = [vp, P(DmmtDeviceFrames), ctypes.c_int, P(DmmtOptions)]
    L.dmmt_encode_striped_device.argtypes = [vp, P(DmmtStripe), ctypes.c_int, P(DmmtOptions), P(vp), P(sz),
                                             P(ctypes.c_uint64)]
    L.dmmt_last_error_detail.argtypes = []
    L.dmmt_last_error_message.argtypes = []
    L.dmmt_last_error_message.restype = ctypes.c_char_p
    L.dmmt_build_info.argtypes = []
    L.dmmt_build_info.restype = ctypes.c_char_p
    _lib = L
    return L


# ---------------------------------------------------------------- C structs

class DmmtImage(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint16), ("height", ctypes.c_uint16), ("maxval", ctypes.c_uint16),
                ("sample_bytes", ctypes.c_uint16), ("rgb", ctypes.c_void_p)]


class DmmtOptions(ctypes.Structure):
    _fields_ = [("subsampling", ctypes.c_int32), ("bits_per_channel", ctypes.c_int32),
                ("luma_q", ctypes.c_uint8 * 64), ("chroma_q", ctypes.c_uint8 * 64),
                ("n_threads", ctypes.c_int32), ("restart_interval", ctypes.c_int32)]


class DmmtDeviceFrames(ctypes.Structure):
    _fields_ = [("d_rgb", ctypes.c_void_p), ("frame_stride", ctypes.c_size_t), ("n_frames", ctypes.c_int32),
                ("width", ctypes.c_uint16), ("height", ctypes.c_uint16), ("maxval", ctypes.c_uint16),
                ("sample_bytes", ctypes.c_uint16), ("d_out", ctypes.c_void_p), ("out_stride", ctypes.c_size_t),
                ("d_out_len", ctypes.c_void_p)]


class DmmtStripe(ctypes.Structure):
    _fields_ = [("d_rgb", ctypes.c_void_p), ("width", ctypes.c_uint16), ("height", ctypes.c_uint16),
                ("maxval", ctypes.c_uint16), ("sample_bytes", ctypes.c_uint16), ("mcu_row0", ctypes.c_int32),
                ("mcu_rows", ctypes.c_int32)]


class DmmtPpmHeader(ctypes.Structure):
    _fields_ = [("width", ctypes.c_uint16), ("height", ctypes.c_uint16), ("maxval", ctypes.c_uint16),
                ("binary", ctypes.c_int32), ("body_offset", ctypes.c_uint64)]


class DmmtPpmFile(ctypes.Structure):
    _fields_ = [("d_text", ctypes.c_void_p), ("len", ctypes.c_size_t), ("header", DmmtPpmHeader),
                ("d_out", ctypes.c_void_p), ("out_capacity", ctypes.c_size_t), ("d_out_len", ctypes.c_void_p)]


STRIPE_HIST_WORDS = 2 * (16 + 256)


def _check(rc: int, what: str = ""):
    if rc != 0:
        raise Error(rc, what)


# ---------------------------------------------------------------- presets / options

class ChromaSubsamplingPreset(enum.IntEnum):
    """src/image/subsampling.rs:11-55"""
    P444 = 0
    P422 = 1
    P420 = 2

    def horizontal_rate(self) -> int:
        return 1 if self == ChromaSubsamplingPreset.P444 else 2

    def vertical_rate(self) -> int:
        return 2 if self == ChromaSubsamplingPreset.P420 else 1


class QuantizationTablePreset(enum.IntEnum):
    """src/image/writer/jpeg/quantization_tables.rs:232-284 (names and aliases)"""
    Specification = 0
    Flat = 1
    MSSIMKodakTuned = 2
    PSNRHVSNKodakTuned = 3
    DCTunePerceptualOptimization = 4
    AVisualDetectionModel = 5
    AnImprovedDetectionModel = 6

    @classmethod
    def from_name(cls, s: str) -> "QuantizationTablePreset":
        names = {
            "Specification": 0, "Spec": 0, "Default": 0, "0": 0, "Flat": 1, "1": 1, "MSSIM-Kodak-Tuned": 2, "2": 2,
            "PSNR-HVS-N-Kodak-Tuned": 3, "4": 3, "DCTune-Perceptual-Optimization": 4, "6": 4,
            "A-visual-detection-model": 5, "7": 5, "An-improved-detection-model": 6, "8": 6,
        }
        if s not in names:
            raise ValueError(f"invalid quantization table preset '{s}'")
        return cls(names[s])

    def to_pair(self):
        """QuantizationTablePreset::to_pair (quantization_tables.rs:286-327): (luma, chroma) natural order."""
        return quantization_preset(int(self))


def quantization_preset(preset: int):
    L = (ctypes.c_uint8 * 64)()
    C = (ctypes.c_uint8 * 64)()
    _check(lib().dmmt_quantization_preset(int(preset), L, C), "quantization preset")
    return list(L), list(C)


def quality_tables(quality: int):
    """Extension: IJG quality scaling of the Annex K tables (q50 == Specification)."""
    L = (ctypes.c_uint8 * 64)()
    C = (ctypes.c_uint8 * 64)()
    _check(lib().dmmt_quality_tables(int(quality), L, C), "quality tables")
    return list(L), list(C)


@dataclass
class JpegTransformationOptions:
    """src/image/writer/jpeg.rs:31-39; tables may be given explicitly (quality extension)."""
    chroma_subsampling_preset: ChromaSubsamplingPreset = ChromaSubsamplingPreset.P420
    bits_per_channel: int = 8
    quantization_table_preset: QuantizationTablePreset = QuantizationTablePreset.Specification
    luma_table: list | None = None
    chroma_table: list | None = None
    restart_interval: int = 0
    number_of_threads: int = 1

    def to_c(self) -> DmmtOptions:
        o = DmmtOptions()
        o.subsampling = int(self.chroma_subsampling_preset)
        o.bits_per_channel = int(self.bits_per_channel)
        if self.luma_table is not None:
            lq, cq = self.luma_table, self.chroma_table
        else:
            lq, cq = QuantizationTablePreset(self.quantization_table_preset).to_pair()
        for i in range(64):
            o.luma_q[i] = int(lq[i])
            o.chroma_q[i] = int(cq[i])
        o.n_threads = int(self.number_of_threads)
        o.restart_interval = int(self.restart_interval)
        return o


# ---------------------------------------------------------------- image

@dataclass
class Image:
    """Image (src/image.rs:7-11).  Integer samples are kept raw with their maxval
    and the GPU applies ``v as f32 / max as f32`` (color.rs:45-53); float32
    samples are the reference's Image<f32> dots, already normalised."""
    width: int
    height: int
    maxval: int
    samples: np.ndarray  # (height, width, 3) uint8, uint16 or float32

    @classmethod
    def from_array(cls, rgb, maxval: int = 255) -> "Image":
        a = np.asarray(rgb)
        if a.ndim != 3 or a.shape[2] != 3:
            raise ValueError("rgb must be (height, width, 3)")
        if a.dtype == np.float32:
            return cls(a.shape[1], a.shape[0], int(maxval), np.ascontiguousarray(a))
        dt = np.uint8 if maxval <= 255 and (a.size == 0 or a.max() <= 255) else np.uint16
        return cls(a.shape[1], a.shape[0], int(maxval), np.ascontiguousarray(a, dtype=dt))

    def to_c(self) -> DmmtImage:
        s = self.samples
        im = DmmtImage()
        im.width, im.height, im.maxval = self.width, self.height, self.maxval
        im.sample_bytes = s.dtype.itemsize
        im.rgb = s.ctypes.data
        return im


def _image_from_c(im: DmmtImage) -> Image:
    n = im.width * im.height * 3
    dt = np.uint8 if im.sample_bytes == 1 else np.uint16
    buf = (ctypes.c_uint8 * (n * im.sample_bytes)).from_address(im.rgb) if n else b""
    arr = np.frombuffer(bytes(buf), dtype=dt).reshape(im.height, im.width, 3).copy()
    lib().dmmt_free(im.rgb)
    return Image(im.width, im.height, im.maxval, arr)


class PPMImageReader:
    """src/image/reader/ppm.rs:9-25 (P3 as the reference; P6 as an extension)."""

    def __init__(self, reader):
        self.reader = reader

    def read_image(self) -> Image:
        data = self.reader.read() if hasattr(self.reader, "read") else bytes(self.reader)
        buf = ctypes.create_string_buffer(data, len(data))
        im = DmmtImage()
        _check(lib().dmmt_parse_ppm(ctypes.cast(buf, ctypes.c_void_p), len(data), ctypes.byref(im)), "read_image")
        return _image_from_c(im)


def parse_ppm_header(data: bytes) -> DmmtPpmHeader:
    """the four header tokens (ppm.rs:145-222) read on the host; body_offset is the
    first byte after the whitespace that ended the max value"""
    buf = ctypes.create_string_buffer(data, len(data))
    h = DmmtPpmHeader()
    _check(lib().dmmt_parse_ppm_header(ctypes.cast(buf, ctypes.c_void_p), len(data), ctypes.byref(h)),
           "parse_ppm_header")
    return h


# ---------------------------------------------------------------- encoder

class Encoder:
    """A GPU context (dmmt_ctx): one device, one stream, pooled workspace.
    Plays the role of the ThreadPool the reference passes around (lib.rs:62).
    ``devices=[...]``: a multi-GPU context (dmmt_ctx_create_multi), one member
    context and host thread per id; encode() then splits the image into MCU-row
    stripes over the members and encode_batch() deals frames round-robin."""

    def __init__(self, device: int = 0, devices=None):
        self._ctx = ctypes.c_void_p()
        if devices is not None:
            ids = (ctypes.c_int * len(devices))(*[int(d) for d in devices])
            _check(lib().dmmt_ctx_create_multi(ids, len(devices), ctypes.byref(self._ctx)),
                   f"dmmt_ctx_create_multi({list(devices)})")
            self.device = int(devices[0]) if len(devices) else 0
        else:
            _check(lib().dmmt_ctx_create(int(device), ctypes.byref(self._ctx)), f"dmmt_ctx_create({device})")
            self.device = device

    def num_devices(self) -> int:
        return lib().dmmt_ctx_num_devices(self._ctx)

    def check_device(self) -> int:
        """dmmt_ctx_check_device: the context's GPU is the working thread's device and
        every pooled buffer lies on it (every member, on its own thread, for a
        multi-GPU context); returns the (first) device id"""
        d = ctypes.c_int32(-1)
        _check(lib().dmmt_ctx_check_device(self._ctx, ctypes.byref(d)), "check_device")
        return int(d.value)

    def member(self, i: int) -> int:
        """member context i's handle (borrowed: valid while this context lives)"""
        return lib().dmmt_ctx_member(self._ctx, int(i)) or 0

    def member_encoder(self, i: int) -> "Encoder":
        """member context i as an Encoder view (device memory, synthetic frames,
        copies on that member's device); borrowed: valid while this context lives,
        and its close() leaves the member alone"""
        h = self.member(i)
        if not h:
            raise Error(-102, f"no member {i}")  # DMMT_E_INVALID_ARGUMENT
        return _MemberView(h, self.device if self.num_devices() == 1 else None)

    def encode_striped(self, image: "Image", options: "JpegTransformationOptions", n_stripes: int = 0) -> bytes:
        """one image as MCU-row stripes over the members (dmmt_jpeg_encode_striped)"""
        im = image.to_c()
        out = ctypes.c_void_p()
        n = ctypes.c_size_t()
        _check(lib().dmmt_jpeg_encode_striped(self._ctx, ctypes.byref(im), ctypes.byref(options.to_c()),
                                              int(n_stripes), ctypes.byref(out), ctypes.byref(n)), "encode_striped")
        data = ctypes.string_at(out.value, n.value)
        lib().dmmt_free(out)
        return data

    def encode_device_multi(self, frames, options: "JpegTransformationOptions"):
        """frames[i]: a DmmtDeviceFrames in member i's HBM; enqueued, see synchronize()"""
        arr = (DmmtDeviceFrames * len(frames))(*frames)
        _check(lib().dmmt_encode_device_multi(self._ctx, arr, len(frames), ctypes.byref(options.to_c())),
               "encode_device_multi")

    def encode_striped_device(self, stripes, options: "JpegTransformationOptions", d_outs, caps):
        """stripes[i] in member i's HBM; returns the byte count written to each d_outs[i]"""
        n = len(stripes)
        st = (DmmtStripe * n)(*stripes)
        outs = (ctypes.c_void_p * n)(*d_outs)
        cp = (ctypes.c_size_t * n)(*caps)
        lens = (ctypes.c_uint64 * n)()
        _check(lib().dmmt_encode_striped_device(self._ctx, st, n, ctypes.byref(options.to_c()), outs, cp, lens),
               "encode_striped_device")
        return [int(x) for x in lens]

    @property
    def handle(self):
        return self._ctx

    def close(self):
        if self._ctx:
            lib().dmmt_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    # -- whole path
    def encode(self, image: Image, options: JpegTransformationOptions) -> bytes:
        return self.encode_batch([image], options)[0]

    def encode_batch(self, images, options: JpegTransformationOptions):
        n = len(images)
        arr = (DmmtImage * n)(*[im.to_c() for im in images])
        outs = (ctypes.c_void_p * n)()
        lens = (ctypes.c_size_t * n)()
        opt = options.to_c()
        _check(lib().dmmt_jpeg_encode_batch(self._ctx, arr, n, ctypes.byref(opt), outs, lens), "encode")
        res = []
        for i in range(n):
            res.append(ctypes.string_at(outs[i], lens[i]))
            lib().dmmt_free(outs[i])
        return res

    # -- stages
    def forward_blocks(self, image: Image, options: JpegTransformationOptions) -> np.ndarray:
        hr = ChromaSubsamplingPreset(options.chroma_subsampling_preset).horizontal_rate()
        vr = ChromaSubsamplingPreset(options.chroma_subsampling_preset).vertical_rate()
        wp = -(-image.width // (8 * hr)) * 8 * hr
        hp = -(-image.height // (8 * vr)) * 8 * vr
        cap = (wp * hp) // 64 * 3
        out = np.zeros((cap, 64), np.int16)
        nb = ctypes.c_size_t()
        opt = options.to_c()
        im = image.to_c()
        _check(lib().dmmt_forward_blocks(self._ctx, ctypes.byref(im), ctypes.byref(opt), out.ctypes.data, cap,
                                         ctypes.byref(nb)), "forward_blocks")
        return out[:nb.value].copy()

    def encode_coefficients(self, coef_zz: np.ndarray, width: int, height: int,
                            options: JpegTransformationOptions) -> bytes:
        c = np.ascontiguousarray(coef_zz, dtype=np.int16)
        out = ctypes.c_void_p()
        n = ctypes.c_size_t()
        opt = options.to_c()
        _check(lib().dmmt_encode_coefficients(self._ctx, c.ctypes.data, c.shape[0], width, height, ctypes.byref(opt),
                                              ctypes.byref(out), ctypes.byref(n)), "encode_coefficients")
        data = ctypes.string_at(out.value, n.value)
        lib().dmmt_free(out)
        return data

    def dct_transform(self, blocks: np.ndarray) -> np.ndarray:
        """Discrete8x8CosineTransformer::transform_on_threadpool (cosine_transform.rs:55-73) on the GPU."""
        a = np.ascontiguousarray(blocks, dtype=np.float32).copy()
        _check(lib().dmmt_dct_transform(self._ctx, a.ctypes.data, a.size), "dct_transform")
        return a

    # -- device resident
    def encode_device(self, d_rgb: int, n_frames: int, width: int, height: int, options: JpegTransformationOptions,
                      d_out: int, out_stride: int, d_out_len: int, frame_stride: int | None = None, maxval: int = 255,
                      sample_bytes: int = 1, stream: int | None = None, opt_c: DmmtOptions | None = None):
        f = DmmtDeviceFrames()
        f.d_rgb = d_rgb
        f.frame_stride = frame_stride if frame_stride is not None else width * height * 3 * sample_bytes
        f.n_frames = n_frames
        f.width, f.height, f.maxval, f.sample_bytes = width, height, maxval, sample_bytes
        f.d_out, f.out_stride, f.d_out_len = d_out, out_stride, d_out_len
        opt = opt_c if opt_c is not None else options.to_c()
        _check(lib().dmmt_encode_device(self._ctx, ctypes.byref(f), ctypes.byref(opt), stream), "encode_device")

    def set_lanes(self, n: int):
        """pipelined device encodes: consecutive encode_device calls with stream None
        go round-robin to n workspaces and streams (include/dmmt_jpeg.h)"""
        _check(lib().dmmt_ctx_set_lanes(self._ctx, n), "set_lanes")

    def synchronize(self):
        _check(lib().dmmt_ctx_synchronize(self._ctx), "synchronize")

    def decode_ppm_device(self, d_text: int, length: int, header: DmmtPpmHeader, d_rgb: int, stream=None):
        """parse_all_dots (ppm.rs:224-252) on the GPU: the whole file at d_text ->
        width*height*3 samples at d_rgb (uint8 if maxval <= 255 else uint16)"""
        _check(lib().dmmt_decode_ppm_device(self._ctx, d_text, length, ctypes.byref(header), d_rgb, stream),
               "decode_ppm_device")

    def convert_ppm_device_batch(self, files, options: JpegTransformationOptions | None = None,
                                 opt_c: DmmtOptions | None = None, check: bool = True):
        """convert_ppm_to_jpeg (lib.rs:59-77) for files already in HBM, pipelined over
        the lanes (dmmt_convert_ppm_device_batch).  files: (d_text, length, header,
        d_out, out_capacity, d_out_len) tuples.  Returns the per-file codes; with
        check, raises the first error."""
        n = len(files)
        arr = (DmmtPpmFile * max(n, 1))()
        for i, (d_text, length, header, d_out, cap, d_len) in enumerate(files):
            arr[i].d_text, arr[i].len, arr[i].header = d_text, length, header
            arr[i].d_out, arr[i].out_capacity, arr[i].d_out_len = d_out, cap, d_len
        codes = (ctypes.c_int32 * max(n, 1))()
        opt = opt_c if opt_c is not None else options.to_c()
        rc = lib().dmmt_convert_ppm_device_batch(self._ctx, arr, n, ctypes.byref(opt), codes)
        if check:
            _check(rc, "convert_ppm_device_batch")
        return [codes[i] for i in range(n)]

    def batch_redone(self) -> int:
        """files the last convert_ppm_device_batch redid on their own (diagnostic)"""
        return lib().dmmt_ctx_batch_redone(self._ctx)

    def read_ppm_device(self, data: bytes) -> Image:
        """PPMImageReader::read_image with the body decoded on the GPU: header on the
        host, file bytes to HBM, samples decoded there and copied back"""
        h = parse_ppm_header(data)
        n = h.width * h.height * 3
        dt = np.uint8 if h.maxval <= 255 else np.uint16
        body = len(data) - h.body_offset  # samples the text can fill (as dmmt_convert_ppm_to_jpeg)
        fit = body // np.dtype(dt).itemsize if h.binary else body // 2 + 1
        d_text = self.malloc(max(len(data), 1))
        d_rgb = self.malloc(max(min(n, fit) * np.dtype(dt).itemsize, 1))
        try:
            if data:
                self.h2d(d_text, np.frombuffer(data, np.uint8))
            self.decode_ppm_device(d_text, len(data), h, d_rgb)
            arr = np.frombuffer(self.d2h(d_rgb, n * np.dtype(dt).itemsize), dt).reshape(h.height, h.width, 3)
        finally:
            self.free(d_text)
            self.free(d_rgb)
        return Image(h.width, h.height, h.maxval, arr.copy())

    def malloc(self, nbytes: int) -> int:
        p = ctypes.c_void_p()
        _check(lib().dmmt_device_malloc(self._ctx, nbytes, ctypes.byref(p)), "malloc")
        return p.value

    def free(self, ptr: int):
        _check(lib().dmmt_device_free(self._ctx, ptr), "free")

    def h2d(self, dst: int, src: np.ndarray):
        s = np.ascontiguousarray(src)
        _check(lib().dmmt_memcpy_h2d(self._ctx, dst, s.ctypes.data, s.nbytes), "h2d")

    def d2h(self, src: int, nbytes: int) -> bytes:
        buf = ctypes.create_string_buffer(nbytes)
        _check(lib().dmmt_memcpy_d2h(self._ctx, ctypes.cast(buf, ctypes.c_void_p), src, nbytes), "d2h")
        return buf.raw

    def fill_synthetic(self, d_rgb: int, width: int, height: int, n_frames: int, first_frame: int = 0,
                       seed: int = 0x9E3779B9):
        _check(lib().dmmt_fill_synthetic(self._ctx, d_rgb, width, height, n_frames, first_frame, seed), "synthetic")

    def fill_synthetic_rows(self, d_rgb: int, width: int, height: int, row0: int, rows: int, frame: int = 0,
                            seed: int = 0x9E3779B9):
        _check(lib().dmmt_fill_synthetic_rows(self._ctx, d_rgb, width, height, row0, rows, frame, seed), "synthetic")

    # ---- one image over several GPUs (extension; include/dmmt_jpeg.h "dmmt_stripe")
    @staticmethod
    def stripe(d_rgb: int, width: int, height: int, mcu_row0: int, mcu_rows: int, maxval: int = 255,
               sample_bytes: int = 1) -> DmmtStripe:
        return DmmtStripe(d_rgb, width, height, maxval, sample_bytes, mcu_row0, mcu_rows)

    @staticmethod
    def stripe_max_bytes(stripe: DmmtStripe, options: JpegTransformationOptions) -> int:
        return lib().dmmt_stripe_max_bytes(ctypes.byref(stripe), ctypes.byref(options.to_c()))

    def stripe_analyze(self, stripe: DmmtStripe, options: JpegTransformationOptions) -> np.ndarray:
        """front half of the stripe; returns its symbol histograms (uint64[544])"""
        h = (ctypes.c_uint64 * STRIPE_HIST_WORDS)()
        _check(lib().dmmt_stripe_analyze(self._ctx, ctypes.byref(stripe), ctypes.byref(options.to_c()), h),
               "stripe_analyze")
        return np.ctypeslib.as_array(h).copy()

    def stripe_encode(self, hist_sum, d_out: int, out_cap: int) -> int:
        """tables from the summed histograms; the stripe's bytes into d_out; returns their count"""
        h = (ctypes.c_uint64 * STRIPE_HIST_WORDS)(*[int(x) for x in hist_sum])
        n = ctypes.c_uint64()
        _check(lib().dmmt_stripe_encode(self._ctx, h, d_out, out_cap, ctypes.byref(n)), "stripe_encode")
        return int(n.value)

    # joined stripes (restart_interval 0, the reference's own stream)
    def stripe_dc_edges(self):
        """(first DC, last DC) per component (Y, Cb, Cr) of the analysed stripe"""
        f, l = (ctypes.c_int16 * 3)(), (ctypes.c_int16 * 3)()
        _check(lib().dmmt_stripe_dc_edges(self._ctx, f, l), "stripe_dc_edges")
        return list(f), list(l)

    @staticmethod
    def stripe_fix_dc_hist(hist, first_dc, prev_last_dc) -> np.ndarray:
        """the stripe's histograms with its first DC differences taken from the previous
        stripe's last DCs instead of 0"""
        h = (ctypes.c_uint64 * STRIPE_HIST_WORDS)(*[int(x) for x in hist])
        lib().dmmt_stripe_fix_dc_hist(h, (ctypes.c_int16 * 3)(*first_dc), (ctypes.c_int16 * 3)(*prev_last_dc))
        return np.ctypeslib.as_array(h).copy()

    def stripe_measure(self, hist_sum, prev_last_dc, d_out: int, out_cap: int):
        """tables from the summed histograms and the stripe's bits; returns (bit count, first 16 bits)"""
        h = (ctypes.c_uint64 * STRIPE_HIST_WORDS)(*[int(x) for x in hist_sum])
        bits, f16 = ctypes.c_uint64(), ctypes.c_uint32()
        _check(lib().dmmt_stripe_measure(self._ctx, h, (ctypes.c_int16 * 3)(*prev_last_dc), d_out, out_cap,
                                         ctypes.byref(bits), ctypes.byref(f16)), "stripe_measure")
        return int(bits.value), int(f16.value)

    def stripe_write(self, bit_offset: int, next_bits: int, next16: int) -> int:
        """the stripe's stuffed bytes (after the header, for the first stripe); returns their count"""
        n = ctypes.c_uint64()
        _check(lib().dmmt_stripe_write(self._ctx, bit_offset, next_bits, next16, ctypes.byref(n)), "stripe_write")
        return int(n.value)

    def set_profiling(self, on: bool):
        _check(lib().dmmt_ctx_set_profiling(self._ctx, 1 if on else 0))

    def profile(self):
        n = lib().dmmt_num_stages()
        ms = (ctypes.c_double * n)()
        cnt = (ctypes.c_int32 * n)()
        _check(lib().dmmt_ctx_profile(self._ctx, ms, cnt, n))
        return {lib().dmmt_stage_name(i).decode(): (ms[i], cnt[i]) for i in range(n)}


def stripe_rows(mcuy: int, world: int, rank: int, rows_per_interval: int = 1):
    """MCU rows [row0, row0 + rows) of rank `rank` when `mcuy` MCU rows are split over
    `world` GPUs in whole restart intervals of `rows_per_interval` rows."""
    units = -(-mcuy // rows_per_interval)
    lo = units * rank // world
    hi = units * (rank + 1) // world
    row0 = lo * rows_per_interval
    return row0, min(hi * rows_per_interval, mcuy) - row0


def stripe_seam(bits, first16, k: int):
    """(B_k, next_bits, next16) of stripe k from every stripe's (bit count, first 16
    bits): its global scan bit offset and the up to 16 scan bits that follow it"""
    b_k = int(sum(bits[:k]))
    have, nxt = 0, 0
    for j in range(k + 1, len(bits)):
        t = min(16 - have, int(bits[j]), 16)
        if t > 0:
            nxt |= ((int(first16[j]) >> (16 - t)) << (16 - have - t))
            have += t
        if have == 16:
            break
    return b_k, have, nxt


def encode_striped(enc: "Encoder", stripe: DmmtStripe, options: JpegTransformationOptions, d_out: int,
                   out_cap: int, group=None):
    """One image over the ranks of a torch.distributed group, one MCU-row stripe per
    rank.  With restart intervals the stripes are independent restart
    segments: the only exchange is an all-reduce of the 544 histogram counters (the
    Huffman tables are global per image) and an all-gather of the stripe sizes.
    Without (restart_interval 0, the reference's own stream) two small all-gathers
    join the seams: the stripes' edge DCs before the all-reduce (the DC predictor runs
    on across a seam) and their (bit count, first 16 bits) before the bytes are
    written (stripe k starts at bit B_k, mid-byte).  Returns (bytes of this stripe in
    d_out, its offset in the file, file size); the stripes concatenated in rank order
    are the JPEG file."""
    import torch
    import torch.distributed as dist
    hist = enc.stripe_analyze(stripe, options)
    on_gpu = dist.get_backend(group) == "nccl"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    world, rank = dist.get_world_size(group), dist.get_rank(group)

    def gather(vals):
        out = torch.zeros(world * len(vals), dtype=torch.int64, device=dev)
        dist.all_gather_into_tensor(out, torch.tensor(vals, dtype=torch.int64, device=dev), group=group)
        return out.cpu().view(world, len(vals)).tolist()

    joined = options.restart_interval == 0
    if joined:  # the DC predictors run on across the seams: exchange the edge DCs first
        first, last = enc.stripe_dc_edges()
        edges = gather(first + last)
        prev = edges[rank - 1][3:] if rank > 0 else [0, 0, 0]
        hist = Encoder.stripe_fix_dc_hist(hist, first, prev)
    t = torch.from_numpy(hist.astype(np.int64)).to(dev)
    dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    if joined:  # the scan runs on across the seams: exchange the stripes' bit counts and heads
        bits, f16 = enc.stripe_measure(t.cpu().numpy().astype(np.uint64), prev, d_out, out_cap)
        seams = gather([bits, f16])
        n = enc.stripe_write(*stripe_seam([b for b, _ in seams], [f for _, f in seams], rank))
    else:
        n = enc.stripe_encode(t.cpu().numpy().astype(np.uint64), d_out, out_cap)
    sizes = torch.zeros(dist.get_world_size(group), dtype=torch.int64, device=dev)
    mine = torch.tensor([n], dtype=torch.int64, device=dev)
    dist.all_gather_into_tensor(sizes, mine, group=group)
    sizes = sizes.cpu().tolist()
    rank = dist.get_rank(group)
    return n, int(sum(sizes[:rank])), int(sum(sizes))


def gather_striped(part, n: int, off: int, total: int, root: int = 0, group=None):
    """The whole JPEG file on rank `root`, from the stripes encode_striped left on
    the ranks (the stripes concatenated in rank order).  Every rank
    sends its n bytes point-to-point straight into their place in root's file buffer;
    with the nccl backend (RCCL) that is a device-to-device copy over xGMI, with
    gloo the tensors are CPU tensors.  part: uint8 tensor whose first n bytes are
    this rank's stripe, on the backend's device.  Returns the file (a uint8 tensor
    of `total` bytes on part's device) on root, None on the other ranks."""
    import torch
    import torch.distributed as dist
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if part.dtype != torch.uint8 or part.dim() != 1 or part.numel() < n:
        raise ValueError("part must be a 1-d uint8 tensor holding at least n bytes")
    # (n, off) of every stripe: root places each one, the others only send
    meta = torch.zeros(2 * world, dtype=torch.int64, device=part.device)
    dist.all_gather_into_tensor(meta, torch.tensor([n, off], dtype=torch.int64, device=part.device), group=group)
    meta = meta.cpu().view(world, 2).tolist()
    if sum(m[0] for m in meta) != total or any(meta[r][1] != sum(m[0] for m in meta[:r]) for r in range(world)):
        raise ValueError("stripe sizes and offsets do not tile the file")

    def peer(r):
        return dist.get_global_rank(group, r) if group is not None else r

    if rank != root:
        if n:
            # complete before returning: the caller may rewrite `part` (the next
            # stripe_encode) as soon as this returns, and with RCCL the send runs on
            # its own stream -- wait for it there, then for that on the host
            dist.isend(part[:n], dst=peer(root), group=group).wait()
            if part.is_cuda:
                torch.cuda.current_stream(part.device).synchronize()
        return None
    out = torch.empty(total, dtype=torch.uint8, device=part.device)
    out[off:off + n].copy_(part[:n])
    reqs = [dist.irecv(out[o:o + k], src=peer(r), group=group)
            for r, (k, o) in enumerate(meta) if r != root and k]
    for q in reqs:
        q.wait()
    return out


def max_jpeg_bytes(width: int, height: int, subsampling: int) -> int:
    return lib().dmmt_max_jpeg_bytes(width, height, int(subsampling))


def device_count() -> int:
    n = ctypes.c_int()
    lib().dmmt_device_count(ctypes.byref(n))
    return n.value



class _MemberView(Encoder):
    """a borrowed member context of a multi-GPU Encoder (Encoder.member_encoder)"""

    def __init__(self, handle: int, device=None):
        self._ctx = ctypes.c_void_p(handle)
        self.device = device

    def close(self):
        pass

class AraiDiscrete8x8CosineTransformer:
    """The reference's pluggable DCT operator (cosine_transform.rs:13-73, arai.rs:95-104), on the GPU."""

    def __init__(self, encoder: Encoder):
        self.encoder = encoder

    def transform(self, block) -> np.ndarray:
        return self.encoder.dct_transform(np.asarray(block, np.float32).reshape(64)).reshape(64)

    def transform_on_threadpool(self, channel: np.ndarray, jobs_chunk_size: int = 700) -> np.ndarray:
        return self.encoder.dct_transform(channel)


class JpegImageWriter:
    """src/image/writer/jpeg.rs:41-75: ``JpegImageWriter::new(writer, image, options, pool).write_image()``."""

    def __init__(self, writer, image: Image, options: JpegTransformationOptions, encoder: Encoder):
        self.writer = writer
        self.image = image
        self.options = options
        self.encoder = encoder

    def write_image(self) -> None:
        data = self.encoder.encode(self.image, self.options)
        try:
            self.writer.write(data)
            if hasattr(self.writer, "flush"):
                self.writer.flush()
        except OSError as e:
            raise Error(-16, str(e)) from e


@dataclass
class Arguments:
    """src/lib.rs:35-42 / cli.rs defaults"""
    input_file: str
    output_file: str
    bits_per_channel: int = 8
    chroma_subsampling_preset: ChromaSubsamplingPreset = ChromaSubsamplingPreset.P420
    number_of_threads: int = 1
    quantization_table_preset: QuantizationTablePreset = QuantizationTablePreset.Specification
    device: int = 0


def convert_ppm_to_jpeg(arguments: Arguments, encoder: Encoder | None = None) -> None:
    """src/lib.rs:59-77"""
    try:
        fin = open(arguments.input_file, "rb")
    except FileNotFoundError as e:
        raise Error(-7, arguments.input_file) from e
    with fin:
        try:
            fout = open(arguments.output_file, "wb")
        except OSError as e:
            raise Error(-8, arguments.output_file) from e
        fout.close()
    # read_image + write_image: the file's bytes go to the GPU as they are, its
    # samples are decoded there (dmmt_decode_ppm_device) and encoded from HBM
    enc = encoder or Encoder(arguments.device)
    opts = JpegTransformationOptions(arguments.chroma_subsampling_preset, arguments.bits_per_channel,
                                     arguments.quantization_table_preset,
                                     number_of_threads=arguments.number_of_threads)
    _check(lib().dmmt_convert_ppm_to_jpeg(enc.handle, os.fsencode(arguments.input_file),
                                          os.fsencode(arguments.output_file), ctypes.byref(opts.to_c())),
           "convert_ppm_to_jpeg")


def encode_array(rgb, maxval: int = 255, subsampling: int = 2, luma=None, chroma=None, preset: int = 0,
                 encoder: Encoder | None = None, bits_per_channel: int = 8) -> bytes:
    """Convenience: one image (HxWx3 array) -> JPEG bytes."""
    enc = encoder or Encoder()
    opts = JpegTransformationOptions(ChromaSubsamplingPreset(subsampling), bits_per_channel,
                                     QuantizationTablePreset(preset), luma, chroma)
    return enc.encode(Image.from_array(rgb, maxval), opts)


__all__ = [
    "Error", "LibraryMissing", "build", "lib", "ChromaSubsamplingPreset", "QuantizationTablePreset",
    "JpegTransformationOptions", "Image", "PPMImageReader", "Encoder", "JpegImageWriter", "Arguments",
    "convert_ppm_to_jpeg", "quantization_preset", "quality_tables", "max_jpeg_bytes", "device_count",
    "DmmtStripe", "stripe_rows", "stripe_seam", "encode_striped",
    "AraiDiscrete8x8CosineTransformer", "encode_array", "io",
]
