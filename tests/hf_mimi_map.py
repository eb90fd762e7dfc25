"""Map the build's Mimi parameter names onto the in-container transformers
``MimiModel`` (an independent PyTorch implementation) so the numpy oracle can
be cross-checked against it.  Test helper only."""
import numpy as np
import torch


def hf_config(m):
    from transformers import MimiConfig
    return MimiConfig(
        hidden_size=m.dimension, num_filters=m.n_filters, upsampling_ratios=list(m.ratios),
        kernel_size=m.kernel_size, residual_kernel_size=m.residual_kernel_size,
        last_kernel_size=m.last_kernel_size, dilation_growth_rate=m.dilation_base, compress=m.compress,
        codebook_size=m.bins, codebook_dim=m.codebook_dim, vector_quantization_hidden_dimension=m.codebook_dim,
        num_quantizers=m.n_q, num_semantic_quantizers=1, upsample_groups=m.dimension,
        num_hidden_layers=m.num_layers, intermediate_size=m.dim_feedforward,
        num_attention_heads=m.num_heads, num_key_value_heads=m.num_heads, head_dim=m.dimension // m.num_heads,
        hidden_act="gelu_pytorch_tanh" if m.gelu == "tanh" else "gelu", sliding_window=m.context,
        rope_parameters={"rope_type": "default", "rope_theta": m.max_period},
        layer_scale_initial_scale=m.layer_scale, norm_eps=m.norm_eps, use_cache=False,
    )


def _rope_perm(hd):
    # interleaved pair (2i, 2i+1) -> rotate_half pair (i, i + hd/2)
    return np.concatenate([np.arange(0, hd, 2), np.arange(1, hd, 2)])


def hf_state_dict(m, w):
    from csm_mlx.weights import mimi_layout
    sd = {}
    enc, dec = mimi_layout(m)
    for side, layout in (("encoder", enc), ("decoder", dec)):
        for kind, p, meta in layout:
            idx = p.split(".")[-1]
            if kind == "conv":
                sd[f"{side}.layers.{idx}.conv.weight"] = w[f"{p}.conv.conv.weight"]
                sd[f"{side}.layers.{idx}.conv.bias"] = w[f"{p}.conv.conv.bias"]
            elif kind == "convtr":
                sd[f"{side}.layers.{idx}.conv.weight"] = w[f"{p}.convtr.convtr.weight"]
                sd[f"{side}.layers.{idx}.conv.bias"] = w[f"{p}.convtr.convtr.bias"]
            else:
                for j in (1, 3):
                    sd[f"{side}.layers.{idx}.block.{j}.conv.weight"] = w[f"{p}.block.{j}.conv.conv.weight"]
                    sd[f"{side}.layers.{idx}.block.{j}.conv.bias"] = w[f"{p}.block.{j}.conv.conv.bias"]
    d, H = m.dimension, m.num_heads
    hd = d // H
    perm = np.concatenate([h * hd + _rope_perm(hd) for h in range(H)])
    for t in ("encoder_transformer", "decoder_transformer"):
        for l in range(m.num_layers):
            p = f"{t}.transformer.layers.{l}"
            q = f"{t}.layers.{l}"
            inp = w[f"{p}.self_attn.in_proj_weight"]
            sd[f"{q}.self_attn.q_proj.weight"] = inp[:d][perm]
            sd[f"{q}.self_attn.k_proj.weight"] = inp[d:2 * d][perm]
            sd[f"{q}.self_attn.v_proj.weight"] = inp[2 * d:]
            sd[f"{q}.self_attn.o_proj.weight"] = w[f"{p}.self_attn.out_proj.weight"]
            sd[f"{q}.input_layernorm.weight"] = w[f"{p}.norm1.weight"]
            sd[f"{q}.input_layernorm.bias"] = w[f"{p}.norm1.bias"]
            sd[f"{q}.post_attention_layernorm.weight"] = w[f"{p}.norm2.weight"]
            sd[f"{q}.post_attention_layernorm.bias"] = w[f"{p}.norm2.bias"]
            sd[f"{q}.mlp.fc1.weight"] = w[f"{p}.linear1.weight"]
            sd[f"{q}.mlp.fc2.weight"] = w[f"{p}.linear2.weight"]
            sd[f"{q}.self_attn_layer_scale.scale"] = w[f"{p}.layer_scale_1.scale"]
            sd[f"{q}.mlp_layer_scale.scale"] = w[f"{p}.layer_scale_2.scale"]
    sd["downsample.conv.weight"] = w["downsample.conv.conv.conv.weight"]
    sd["upsample.conv.weight"] = w["upsample.convtr.convtr.convtr.weight"]
    for ours, theirs, nq in (("rvq_first", "semantic_residual_vector_quantizer", 1),
                             ("rvq_rest", "acoustic_residual_vector_quantizer", m.n_q - 1)):
        sd[f"quantizer.{theirs}.input_proj.weight"] = w[f"quantizer.{ours}.input_proj.weight"]
        sd[f"quantizer.{theirs}.output_proj.weight"] = w[f"quantizer.{ours}.output_proj.weight"]
        for k in range(nq):
            sd[f"quantizer.{theirs}.layers.{k}.codebook.embed_sum"] = w[f"quantizer.{ours}.vq.layers.{k}._codebook.embedding_sum"]
            sd[f"quantizer.{theirs}.layers.{k}.codebook.cluster_usage"] = w[f"quantizer.{ours}.vq.layers.{k}._codebook.cluster_usage"]
    return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in sd.items()}


def build_hf_mimi(m, w):
    from transformers import MimiModel
    cfg = hf_config(m)
    cfg._attn_implementation = "eager"
    model = MimiModel(cfg).eval()
    sd = hf_state_dict(m, w)
    missing, unexpected = model.load_state_dict(sd, strict=False)
    missing = [k for k in missing if not k.endswith(".initialized")]
    assert not unexpected, unexpected
    assert not missing, missing
    return model
