python tools/sss_shard_rehearsal.py --sizes 200
