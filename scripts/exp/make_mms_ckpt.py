"""Write a random-weight checkpoint of the MMS-TTS shape (transformers'
VitsConfig defaults) + a 38-character vocab.json into DIR (for served-hub
runs with HUB_TTS_CHECKPOINT)."""
import json
import os
import sys

import torch
from transformers import VitsConfig, VitsModel

d = sys.argv[1]
os.makedirs(d, exist_ok=True)
torch.manual_seed(0)
VitsModel(VitsConfig()).save_pretrained(d, safe_serialization=True)
with open(os.path.join(d, "vocab.json"), "w") as f:
    json.dump({c: i for i, c in enumerate("_ '-abcdefghijklmnopqrstuvwxyz0123456")}, f)
print("checkpoint", d)
