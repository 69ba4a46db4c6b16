"""CPU restatement of the crdt merge path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this package; crdt_amd never does.  See crdt_oracle.h for parity status.
"""
