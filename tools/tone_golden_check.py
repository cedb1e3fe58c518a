import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np, torch
from tests.conftest import load_golden
from oracle import stoi_oracle
from fast_speech_enhancement_metrics_amd import STOI
g = load_golden('tones_10k')
s, e = STOI(10000, use_gpu=True).scores(torch.from_numpy(g['clean_f']).cuda(), torch.from_numpy(g['noisy_f']).cuda())
s, e = s.cpu().numpy(), e.cpu().numpy()
so, eo = stoi_oracle.stoi(g['clean_f'], g['noisy_f'], 10000)
print('ref   ', np.round(g['stoi'], 5), np.round(g['estoi'], 5))
print('engine', np.round(s, 5), np.round(e, 5))
print('engine-ref max', np.max(abs(s - g['stoi'])), np.max(abs(e - g['estoi'])))
print('oracle-ref max', np.max(abs(so - g['stoi'])), np.max(abs(eo - g['estoi'])))
