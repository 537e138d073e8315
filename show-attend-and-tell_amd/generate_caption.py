"""Caption one image with beam search (reference: generate_caption.py) on the MI355X path.

    python show-attend-and-tell_amd/generate_caption.py --img-path dog.jpg --model model/model_vgg19_5.pth
    python show-attend-and-tell_amd/generate_caption.py --img-path dog.jpg --model m.pth --plot att.png

Same flags as the reference (generate_caption.py:153-160) plus:
  --model-config  model_config.json written by train.py (default: next to --model); the
                  reference reads network / data / ado / bert / attention from it (:39-47)
  --beam-size     beam width (the reference hard-codes 3, :81)
  --dtype         fp32 (default, reference numerics) | bf16
  --bert-vocab    a local bert-base-uncased vocab.txt (offline BertTokenizer); without it BERT
                  ids print as the [CLS]/[SEP]/[PAD]/tokN stub
  --plot          write the attention visualisation (:111-150) to this PNG (matplotlib)
  --encoder-weights  the trunk's state_dict (weights_only); default: the encoder_weights entry
                  train.py wrote into model_config.json.  The reference relies on torchvision's
                  pretrained weights being the same everywhere; this build has none offline, so the
                  trunk must be the one the decoder was trained on
W&B restore (--wandb-run/--wandb-model) needs network access and is not supported here.
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

if __package__ in (None, ""):
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import sat_amd  # noqa: E402

MEAN = np.array([0.485, 0.456, 0.406], dtype=np.float32)   # train.py:27-32
STD = np.array([0.229, 0.224, 0.225], dtype=np.float32)


def load_image(path):
    """pil_loader + data_transforms (dataset.py:9-12, train.py:27-32) -> [1, 3, 224, 224]."""
    from PIL import Image
    with open(path, "rb") as f:
        img = Image.open(f).convert("RGB").resize((224, 224), Image.BILINEAR)
    x = (np.asarray(img, dtype=np.float32) / 255.0 - MEAN) / STD
    return torch.from_numpy(x.transpose(2, 0, 1).copy()).unsqueeze(0)


def load_model(model_path, model_config_path=None, dtype=torch.float32, device="cuda", bert_vocab=None,
               encoder_weights=None):
    """generate_caption.py:24-75: config -> Encoder/Decoder, checkpoint loaded (strict, then lax); the
    encoder trunk from ``encoder_weights`` or the config's ``encoder_weights`` entry (train.py)."""
    if model_path is None:
        raise ValueError("Model path must be provided (W&B restore is not available offline)")
    model_config_path = model_config_path or os.path.join(os.path.dirname(model_path) or ".", "model_config.json")
    with open(model_config_path) as f:
        cfg = json.load(f)
    sd = torch.load(model_path, map_location="cpu", weights_only=True)
    tokenizer = None
    if cfg["bert"]:
        if bert_vocab:
            from transformers import BertTokenizer
            tokenizer = BertTokenizer(bert_vocab)
        vocab = sd["embedding.weight"].shape[0]
        word_dict = None
    else:
        word_dict = json.load(open(os.path.join(cfg["data"], "word_dict.json")))
        vocab = len(word_dict)
    encoder = sat_amd.Encoder(cfg["network"], dtype=dtype)
    enc_w = encoder_weights or cfg.get("encoder_weights")
    if enc_w and not os.path.exists(enc_w):
        # the model directory was copied or moved (train.py records an absolute path): the weights sit
        # next to model_config.json
        enc_w = os.path.join(os.path.dirname(model_config_path) or ".", os.path.basename(enc_w))
    if enc_w:
        encoder.load_state_dict(torch.load(enc_w, map_location="cpu", weights_only=True))
    else:
        print("WARNING: no encoder weights (neither --encoder-weights nor model_config.json's encoder_weights): "
              "the trunk is randomly initialised and its features do not match the ones the decoder was trained "
              "on", file=sys.stderr, flush=True)
    decoder = sat_amd.Decoder(vocab, encoder.dim, ado=cfg["ado"], bert=cfg["bert"], attention=cfg["attention"],
                              bert_embedding_weight=sd.get("embedding.weight") if cfg["bert"] else None,
                              tokenizer=tokenizer)
    try:
        decoder.load_state_dict(sd)
    except RuntimeError:
        print("Strict loading failed, loading with strict=False")
        decoder.load_state_dict(sd, strict=False)
    return encoder.to(device).eval(), decoder.to(device).eval(), cfg, word_dict


def caption_image(img, encoder, decoder, beam_size=3):
    """generate_caption.py:84-88: encode, expand to beam rows, beam search."""
    with torch.no_grad():
        feats = encoder(img.to(next(iter(decoder.parameters())).device))
        feats = feats.expand(beam_size, feats.size(1), feats.size(2))
        return decoder.caption(feats, beam_size)


def sentence_tokens(sentence, decoder, word_dict):
    """generate_caption.py:90-101."""
    if decoder.use_bert:
        tok = decoder.tokenizer
        if hasattr(tok, "decode"):
            return tok.decode(sentence, skip_special_tokens=False).split()
        return tok.convert_tokens_to_string(tok.convert_ids_to_tokens(sentence)).split()
    token_dict = {idx: word for word, idx in word_dict.items()}
    out = []
    for idx in sentence:
        out.append(token_dict.get(idx, "<unk>"))
        if idx == word_dict["<eos>"]:
            break
    return out


def plot_attention(img_path, tokens, alpha, network, out_png):
    """generate_caption.py:103-150 (bilinear upsampling in place of skimage's pyramid_expand)."""
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    from PIL import Image
    img = Image.open(img_path)
    w, h = img.size
    if w > h:
        w, h = w * 256 / h, 256
    else:
        w, h = 256, h * 256 / w
    left, top = (w - 224) / 2, (h - 224) / 2
    img = np.asarray(img.resize((int(w), int(h)), Image.BICUBIC).crop((left, top, left + 224, top + 224))
                     .convert("RGB"), dtype=np.float32) / 255
    side = 14 if network == "vgg19" else 7
    alpha = torch.as_tensor(np.asarray(alpha, dtype=np.float32))
    rows = int(np.ceil((len(tokens) + 3) / 4.0))
    plt.figure(figsize=(3 * rows, 12))
    plt.subplot(4, rows, 1)
    plt.imshow(img)
    plt.axis("off")
    for i, word in enumerate(tokens):
        if i >= alpha.shape[0]:
            break
        plt.subplot(4, rows, i + 2)
        plt.text(0, 1, word, backgroundcolor="white", fontsize=13)
        plt.imshow(img)
        a = torch.nn.functional.interpolate(alpha[i].reshape(1, 1, side, side), size=(224, 224), mode="bilinear",
                                            align_corners=False)[0, 0].numpy()
        plt.imshow(a, alpha=0.8, cmap="Greys_r")
        plt.axis("off")
    plt.savefig(out_png, bbox_inches="tight")


def main(argv=None):
    p = argparse.ArgumentParser(description="Show, Attend and Tell Caption Generator (MI355X)")
    p.add_argument("--img-path", type=str, help="path to image")
    p.add_argument("--model", type=str, help="path to model parameters")
    p.add_argument("--wandb-run", type=str, default=None)
    p.add_argument("--wandb-model", type=str, default=None)
    p.add_argument("--model-config", type=str, default=None)
    p.add_argument("--beam-size", type=int, default=3)
    p.add_argument("--dtype", choices=["fp32", "bf16"], default="fp32")
    p.add_argument("--bert-vocab", type=str, default=None)
    p.add_argument("--plot", type=str, default=None)
    p.add_argument("--encoder-weights", type=str, default=None)
    args = p.parse_args(argv)
    if args.wandb_run or args.wandb_model:
        p.error("W&B restore needs network access; pass --model/--model-config")
    dt = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    encoder, decoder, cfg, word_dict = load_model(args.model, args.model_config, dt, bert_vocab=args.bert_vocab,
                                                  encoder_weights=args.encoder_weights)
    sentence, alpha = caption_image(load_image(args.img_path), encoder, decoder, args.beam_size)
    tokens = sentence_tokens(sentence, decoder, word_dict)
    print(json.dumps({"caption": " ".join(tokens), "ids": sentence, "score": decoder.last_caption_score}))
    if args.plot:
        plot_attention(args.img_path, tokens, alpha, cfg["network"], args.plot)
    return 0


if __name__ == "__main__":
    sys.exit(main())
