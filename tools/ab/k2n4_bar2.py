"""Patch (tools/build_patched.sh): the N4 narrow K2's compiler barrier after every second k-step (pairs of k-steps'
reads may merge into ds_read2st64_b64 and run one step ahead)."""
k = open("sysid_kernels.h").read()
old = '''          asm volatile("" ::: "memory");
        }
      }
    };'''
assert k.count(old) == 1
k = k.replace(old, '''          if ((kk & 4) != 0) asm volatile("" ::: "memory");
        }
      }
    };''')
open("sysid_kernels.h", "w").write(k)
