"""``deepspeed.ops.op_builder`` import path (reference op_builder/*).

The reference JIT-compiles each op on first use (torch cpp_extension, hipify on ROCm). Here every kernel is
compiled ahead of time for gfx950 by ops/build.py into two in-tree libraries (HIP kernels / host runtime),
so a builder only checks compatibility and returns the loaded module that exposes the op's API."""


class OpBuilder:
    NAME = "op"

    def __init__(self, name=None):
        self.name = name or self.NAME

    def is_compatible(self, verbose=False):
        return True

    def absolute_name(self):
        return f"hcache_deepspeed_amd.ops.{self.name}"

    def load(self, verbose=False):
        raise NotImplementedError


class _Namespace:

    def __init__(self, **kw):
        self.__dict__.update(kw)


class AsyncIOBuilder(OpBuilder):
    NAME = "async_io"

    def load(self, verbose=False):
        from ..aio import aio_handle
        return _Namespace(aio_handle=aio_handle)


class GDSBuilder(AsyncIOBuilder):
    NAME = "gds"

    def load(self, verbose=False):
        from ..aio import aio_handle
        return _Namespace(gds_handle=aio_handle, aio_handle=aio_handle)


class CPUAdamBuilder(OpBuilder):
    NAME = "cpu_adam"

    def load(self, verbose=False):
        from .. import native
        return native.host_lib()


class CPUAdagradBuilder(CPUAdamBuilder):
    NAME = "cpu_adagrad"


class CPULionBuilder(CPUAdamBuilder):
    NAME = "cpu_lion"


class FusedAdamBuilder(OpBuilder):
    NAME = "fused_adam"

    def load(self, verbose=False):
        from .. import native
        return native.kernels()


class FusedLambBuilder(FusedAdamBuilder):
    NAME = "fused_lamb"


class FusedLionBuilder(FusedAdamBuilder):
    NAME = "fused_lion"


class QuantizerBuilder(FusedAdamBuilder):
    NAME = "quantizer"


class FPQuantizerBuilder(FusedAdamBuilder):
    NAME = "fp_quantizer"


class TransformerBuilder(FusedAdamBuilder):
    NAME = "transformer"


class InferenceBuilder(FusedAdamBuilder):
    NAME = "transformer_inference"


class RaggedOpsBuilder(FusedAdamBuilder):
    NAME = "ragged_device_ops"


class RandomLTDBuilder(FusedAdamBuilder):
    NAME = "random_ltd"


class SparseAttnBuilder(FusedAdamBuilder):
    NAME = "sparse_attn"


class EvoformerAttnBuilder(FusedAdamBuilder):
    NAME = "evoformer_attn"


class SpatialInferenceBuilder(FusedAdamBuilder):
    NAME = "spatial_inference"


ALL_OPS = {c.NAME: c for c in (AsyncIOBuilder, GDSBuilder, CPUAdamBuilder, CPUAdagradBuilder, CPULionBuilder,
                               FusedAdamBuilder, FusedLambBuilder, FusedLionBuilder, QuantizerBuilder,
                               FPQuantizerBuilder, TransformerBuilder, InferenceBuilder, RaggedOpsBuilder,
                               RandomLTDBuilder, SparseAttnBuilder, EvoformerAttnBuilder, SpatialInferenceBuilder)}
