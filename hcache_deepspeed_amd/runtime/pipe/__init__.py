from .module import LayerSpec, PipelineModule, TiedLayerSpec  # noqa: F401
