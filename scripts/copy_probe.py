import sys; sys.path.insert(0, "deepflame-dev_amd")
from dfmi.lib import Context
c = Context(0)
for g in (1.0, 4.0, 8.0):
    print(g, c.hbm_copy_peak(g, 20))
