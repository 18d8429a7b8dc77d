"""emurx — MI355X-native TRex-EMU receive path (parse + Namespace/Client classify).

Host-side Python surface over the C-ABI in include/emu_rx.h:
  emurx.abi     ctypes binding, record/descriptor dtypes, constants
  emurx.frames  gopacket-equivalent frame builders (KAT and edge-case frames)
  emurx.synth   seeded synthetic workloads of BASELINE.json configs B-E
  emurx.rx      RxPath: tables + host/device batch entry points (mirrors Parser/VethIFZmq)
"""
from . import abi, frames  # noqa: F401
