import sys, os, numpy as np, torch
sys.path.insert(0, 'ofdm-based-systems_amd'); sys.path.insert(0, 'oracle'); sys.path.insert(0, 'tests')
from ofdm_based_systems import _backend as B
from ofdm_based_systems.engine import LinkEngine, new_stats
import ofdm_oracle as O
cfg = sys.argv[1]
S = int(sys.argv[2])
N, M, ch = {'e': (4096, 256, 'Lin-Phoong_P1'), 'c': (1024, 64, 'severe_multipath'), 'd': (2048, 64, 'Lin-Phoong_P1')}[cfg]
h = np.load('config/channel_models/%s.npy' % ch)
eng = LinkEngine(N, len(h) - 1, h, B.EQ_MMSE, [O.qam_lut(M)], None, B.OFDM_F64)
st = eng.stream()
def tx(sym0, n, y):
    s = new_stats('cuda'); eng.tx(st, None, 7, sym0, n, y, s); torch.cuda.synchronize(); return s.cpu().numpy()
ys = []
for k in range(2):
    y = torch.empty((S, eng.ystride), dtype=eng.cdtype, device='cuda'); tx(0, S, y); ys.append(y)
for k in range(2):
    y = torch.empty((S, eng.ystride), dtype=eng.cdtype, device='cuda'); hh = S // 2
    tx(0, hh, y[:hh]); tx(hh, S - hh, y[hh:]); ys.append(y)
names = ['one1', 'one2', 'half1', 'half2']
for a in range(4):
    for b in range(a + 1, 4):
        d = (ys[a] != ys[b]).any(dim=1).nonzero().flatten().cpu().numpy()
        print(cfg, os.environ.get('OFDM_LIB_VARIANT'), names[a], names[b], 'rows differing', len(d), d[:8])
        if len(d) and a == 0:
            r = int(d[0]); cols = (ys[a][r] != ys[b][r]).nonzero().flatten().cpu().numpy()
            print('   row', r, 'cols', len(cols), cols[:16])
            va, vb = ys[a][r].cpu().numpy(), ys[b][r].cpu().numpy()
            for c in cols[:3]:
                # where else does each value occur (same row, previous row)?
                wa = np.nonzero(np.isclose(ys[a][r - 1].cpu().numpy(), va[c]) | np.isclose(va, va[c]))[0][:6]
                wb = np.nonzero(np.isclose(ys[b][r - 1].cpu().numpy(), vb[c]) | np.isclose(vb, vb[c]))[0][:6]
                print('   col', c, names[a], va[c], 'also at', wa, '|', names[b], vb[c], 'also at', wb)
