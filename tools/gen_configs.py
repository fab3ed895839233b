"""Emit config/<dataset>/{preprocess,model,train}.yaml.

Same key schema as the reference's YAMLs so reference configs
load unchanged; paths are repo-relative and each train.yaml gains an `mi355x:`
block.  Run: python tools/gen_configs.py
"""
import copy
import os
import yaml

ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "config")

def stft_block():
    return {"filter_length": 1024, "hop_length": 256, "win_length": 1024}

def preprocess(name, lang="en", cleaners=("english_cleaners",), pitch="phoneme_level", energy="phoneme_level",
               norm=True):
    return {
        "dataset": name,
        "path": {
            "corpus_path": f"./data/corpus/{name}",
            "lexicon_path": "lexicon/pinyin-lexicon-r.txt" if lang == "zh" else "lexicon/librispeech-lexicon.txt",
            "raw_path": f"./raw_data/{name}",
            "preprocessed_path": f"./preprocessed_data/{name}",
        },
        "preprocessing": {
            "val_size": 512,
            "text": {"text_cleaners": list(cleaners), "language": lang},
            "audio": {"sampling_rate": 22050, "max_wav_value": 32768.0},
            "stft": stft_block(),
            "mel": {"n_mel_channels": 80, "mel_fmin": 0, "mel_fmax": 8000},
            "pitch": {"feature": pitch, "normalization": norm},
            "energy": {"feature": energy, "normalization": norm},
        },
    }

def model(dec_layers=6, pitch_q="linear", multi=False, vocoder_spk="LJSpeech", ref_enc=False, gst=False):
    m = {
        "transformer": {
            "encoder_layer": 4, "encoder_head": 2, "encoder_hidden": 256,
            "decoder_layer": dec_layers, "decoder_head": 2, "decoder_hidden": 256,
            "conv_filter_size": 1024, "conv_kernel_size": [9, 1],
            "encoder_dropout": 0.2, "decoder_dropout": 0.2,
        },
        "variance_predictor": {"filter_size": 256, "kernel_size": 3, "dropout": 0.5},
        "variance_embedding": {"pitch_quantization": pitch_q, "energy_quantization": "linear", "n_bins": 256},
        "multi_speaker": multi,
        "max_seq_len": 1000,
        "vocoder": {"model": "HiFi-GAN", "speaker": vocoder_spk},
    }
    if ref_enc:
        m["reference_encoder"] = {
            "encoder_layer": 4, "encoder_head": 8, "encoder_hidden": 256,
            "conv_layer": 3, "conv_filter_size": 1024, "conv_kernel_size": 3, "dropout": 0.1,
        }
    m["gst"] = {
        "use_gst": gst, "conv_filters": [32, 32, 64, 64, 128, 128], "gru_hidden": 128,
        "token_size": 128, "n_style_token": 10, "attn_head": 4,
    }
    return m

def train(name, batch, total=900000, save=10000, init_lr=None, style=False, anneal=([300000, 400000, 500000], 0.3)):
    t = {
        "ignore_layers": [],
        "path": {
            "ckpt_path": f"./output/ckpt/{name}",
            "log_path": f"./output/log/{name}",
            "result_path": f"./output/result/{name}",
        },
        "optimizer": {
            "batch_size": batch, "betas": [0.9, 0.98], "eps": 1.0e-9, "weight_decay": 0.0,
            "grad_clip_thresh": 1.0, "grad_acc_step": 1, "warm_up_step": 4000,
            "anneal_steps": list(anneal[0]), "anneal_rate": anneal[1],
        },
        "step": {"total_step": total, "log_step": 100, "synth_step": 1000, "val_step": 1000, "save_step": save},
        "mi355x": {"dtype": "bf16", "bucket_mb": 32, "seed": 1234, "num_workers": 4},
    }
    if init_lr is not None:
        t["optimizer"]["init_lr"] = init_lr[0]
        t["optimizer"]["anneal_lr"] = init_lr[1]
    if style:
        t["loss"] = {"lambda_f": 0.001, "anneal_steps": 10000}
    return t

SETS = {
    "LJSpeech": (preprocess("LJSpeech"), model(), train("LJSpeech", 200, save=1000)),
    # reference config/LJSpeech_paper/{preprocess,train}.yaml: frame-level, unnormalised pitch / energy
    # (log pitch bins over Hz), no LR annealing
    "LJSpeech_paper": (preprocess("LJSpeech_paper", pitch="frame_level", energy="frame_level", norm=False),
                       model(dec_layers=4, pitch_q="log"),
                       train("LJSpeech_paper", 48, total=160000, anneal=([], 1.0))),
    "LibriTTS": (preprocess("LibriTTS"), model(multi=True, vocoder_spk="universal"), train("LibriTTS", 16, save=100000)),
    "AISHELL3": (preprocess("AISHELL3", lang="zh", cleaners=()), model(multi=True, vocoder_spk="universal"),
                 train("AISHELL3", 16, save=100000)),
    "BC2013": (preprocess("BC2013"), model(ref_enc=True), train("BC2013", 75, init_lr=(1e-4, 1e-3), style=True)),
    "BC2013_GST": (preprocess("BC2013"), model(gst=True), train("BC2013_GST", 75, init_lr=(1e-4, 1e-3), style=True)),
}
SETS["LJSpeech"][0]["path"]["preprocessed_path"] = "./preprocessed_data/LJSpeech"
SETS["LJSpeech_paper"][0]["path"]["raw_path"] = "./raw_data/LJSpeech"  # shares LJSpeech's aligned corpus

if __name__ == "__main__":
    for name, trip in SETS.items():
        d = os.path.join(ROOT, name)
        os.makedirs(d, exist_ok=True)
        for fname, obj in zip(("preprocess", "model", "train"), trip):
            with open(os.path.join(d, fname + ".yaml"), "w") as f:
                f.write(f"# {name} {fname} config (generated by tools/gen_configs.py)\n")
                yaml.safe_dump(obj, f, sort_keys=False, default_flow_style=None)
    print("wrote", sorted(SETS))
