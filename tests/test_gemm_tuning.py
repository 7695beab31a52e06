"""The shipped TunableOp results (ops/tuned/gemm_gfx950.csv, ops/gemm_tuning.py): it parses, pins
the stack it was measured on, covers the BERT-base GEMM shapes, and loading it is a no-op off-GPU."""
from determined_1_amd.ops import gemm_tuning


def test_shipped_file_lists_the_bert_shapes_and_validators():
    e = gemm_tuning.entries()
    assert len(e) >= 12
    # BERT-base SQuAD bs12 x 384: the QKV / FFN forward and the token-reduction weight gradients
    for key in ("GemmAndBiasTunableOp_BFloat16_TN,tn_2304_4608_768_ld_768_768_2304",
                "GemmTunableOp_BFloat16_NT,nt_3072_768_4608_ld_3072_768_3072"):
        assert key in e, key
    with open(gemm_tuning.SHIPPED) as f:
        validators = {ln.split(",")[1] for ln in f if ln.startswith("Validator")}
    assert {"PT_VERSION", "HIPBLASLT_VERSION", "ROCBLAS_VERSION", "GCN_ARCH_NAME"} <= validators


def test_enable_is_opt_in_and_a_no_op_without_a_gpu(monkeypatch):
    monkeypatch.setitem(gemm_tuning._STATE, "loaded", None)
    monkeypatch.delenv("DET_TUNED_GEMMS", raising=False)
    assert gemm_tuning.enable() is False
    monkeypatch.setitem(gemm_tuning._STATE, "loaded", None)
    monkeypatch.setenv("DET_TUNED_GEMMS", "1")
    monkeypatch.setattr(gemm_tuning.torch.cuda, "is_available", lambda: False)
    assert gemm_tuning.enable() is False
