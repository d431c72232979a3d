"""Correlation modules — drop-in for src/models/common/corr/__init__.py:7-49 (make_cmod, make_flow_regression)."""

from . import dicl, dicl_1x1, dicl_emb, dot  # noqa: F401


def make_cmod(type, feature_dim, radius, dap_init="identity", norm_type="batch", relu_inplace=True, **kwargs):
    if type == "dicl":
        return dicl.CorrelationModule(feature_dim=feature_dim, radius=radius, dap_init=dap_init,
                                      norm_type=norm_type, relu_inplace=relu_inplace, **kwargs)
    if type == "dicl-1x1":
        return dicl_1x1.CorrelationModule(feature_dim=feature_dim, radius=radius, dap_init=dap_init,
                                          norm_type=norm_type, relu_inplace=relu_inplace, **kwargs)
    if type == "dicl-emb":
        return dicl_emb.CorrelationModule(feature_dim=feature_dim, radius=radius, dap_init=dap_init,
                                          norm_type=norm_type, relu_inplace=relu_inplace, **kwargs)
    if type == "dot":
        return dot.CorrelationModule(radius=radius, dap_init=dap_init, **kwargs)
    raise ValueError(f"unknown correlation module type '{type}'")


def make_flow_regression(cmod_type, type, radius, **kwargs):
    from ..heads import make_corr_flow_regression
    return make_corr_flow_regression(cmod_type, type, radius, **kwargs)
