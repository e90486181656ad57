"""Debug: incremental add at the filter_test shape with the old filter given as (a) the built
batch, (b) a probe-only batch imported device-to-device, (c) imported from host bytes."""
import sys, os
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np, torch
from splinterdb_amd import engine as E, keys as K
from oracle import oracle as O
cfg = E.routing_config_init(); ocfg = O.make_config()
for nf in (20000, 1_048_575):
    h0 = O.hash_fixed(K.ids_keys(np.arange(nf, dtype=np.uint64)).reshape(-1), 24)
    h1 = O.hash_fixed(K.ids_keys(2 * np.arange(nf, dtype=np.uint64)).reshape(-1), 24)
    of0 = O.filter_add(ocfg, h0); of1 = O.filter_add(ocfg, h1, value=1, old=of0)
    b0 = E.FilterBatch(cfg, [nf], [0]); b0.build_hashes(torch.from_numpy(h0.view(np.int32)).cuda())
    inf = b0.info(0)
    dp, ds = __import__('ctypes').c_void_p(), __import__('ctypes').c_void_p()
    E.load_library().rf_amd_batch_image_ptrs(b0.h, 0, __import__('ctypes').byref(dp), __import__('ctypes').byref(ds))
    imp_d = E.FilterBatch.imported(cfg, [inf], dp.value, ds.value, device_resident=True)
    img0 = b0.image(0)
    imp_h = E.FilterBatch.imported(cfg, [inf], img0.pages, img0.slots, device_resident=False)
    for name, old in (("built", b0), ("import_d2d", imp_d), ("import_host", imp_h)):
        b1 = E.FilterBatch(cfg, [nf], [1], old=[(old, 0)])
        b1.build_hashes(torch.from_numpy(h1.view(np.int32)).cuda())
        im = b1.image(0)
        print(nf, name, im.num_unique, of1.num_unique, (im.pages.size == of1.pages().size) and bool((im.pages == of1.pages()).all()), flush=True)
