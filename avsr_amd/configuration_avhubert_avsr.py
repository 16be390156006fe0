"""AVHubertAVSRConfig — drop-in for src/avhubert_avsr/configuration_avhubert_avsr.py:15-369.

Same `model_type` ("avhubert_avsr") and the same field names / defaults for every field
the hot path reads, so a reference `config.json` loads unchanged (unknown keys are kept
as attributes by PretrainedConfig, as in the reference).
"""
from transformers.configuration_utils import PretrainedConfig

# (field, default) pairs the AVSR hot path reads; defaults as configuration_avhubert_avsr.py
_FIELDS = dict(
    odim=5049, adim=1024, ddim=1024, dheads=16, dunits=3072, dlayers=6,
    dropout_rate=0.1, transformer_attn_dropout_rate=0.1, lsm_weight=0.1,
    transformer_length_normalized_loss=False, mtlalpha=0.1, ctc_type="builtin",
    hidden_size=1024, num_attention_heads=16, intermediate_size=4096, num_hidden_layers=24,
    hidden_act="gelu", layer_norm_eps=1e-5, hidden_dropout=0.1, attention_dropout=0.1,
    activation_dropout=0.0, layerdrop=0.0, num_conv_pos_embeddings=128,
    num_conv_pos_embedding_groups=16, feat_extract_activation="gelu",
    audio_feat_dim=104, encoder_embed_dim=1024, feature_grad_mult=0.1,
    modality_dropout=0.5, audio_dropout=0.5, modality_fuse="concat", modality="av",
    dropout_input=0.1, dropout_features=0.1, masking_type="input", num_classes=2004,
    final_dim=256, resnet_relu_type="prelu", resnet_weights=None, untie_final_proj=True,
    # fields the reference declares but the fine-tune path never reads (kept for config.json parity)
    aheads=12, eunits=3072, elayers=12, transformer_input_layer="conv3d",
    transformer_encoder_attn_layer_type="rel_mha", macaron_style=True, use_cnn_module=True,
    cnn_module_kernel=31, zero_triu=False, a_upsample_ratio=1, relu_type="swish",
    rel_pos_type="latest", fusion_hdim=8192, fusion_norm="batchnorm", label_rate=25,
    sample_rate=25, sub_encoder_layers=0, logit_temp=0.1, sim_type="cosine",
)


class AVHubertAVSRConfig(PretrainedConfig):
    model_type = "avhubert_avsr"

    def __init__(self, **kwargs):
        for k, v in _FIELDS.items():
            setattr(self, k, kwargs.pop(k, v))
        super().__init__(**kwargs)
