// objpool.h -- per-thread recycling of the control plane's fixed-size heap
// objects (window subwindows, recovery-list nodes).  A bench step creates and
// frees thousands of codecs, each owning dozens of these; recycling them keeps
// the C heap (whose cross-thread frees contend on its arena locks) out of the
// hot path.  An object freed on one thread is reused by that thread.
#pragma once

#include <cstddef>
#include <vector>

namespace sgpu {

template <class T>
class ObjPool
{
public:
    static T* get()
    {
        Stash& s = stash();
        if (!s.items.empty()) {
            T* p = s.items.back();
            s.items.pop_back();
            return p;
        }
        return new T;
    }
    /// `p` must already be in its freshly constructed state.
    static void put(T* p)
    {
        Stash& s = stash();
        if (s.items.size() < kMax)
            s.items.push_back(p);
        else
            delete p;
    }

private:
    static constexpr size_t kMax = 1u << 14;
    struct Stash
    {
        std::vector<T*> items;
        ~Stash()
        {
            for (T* p : items)
                delete p;
        }
    };
    static Stash& stash()
    {
        thread_local Stash s;
        return s;
    }
};

} // namespace sgpu
