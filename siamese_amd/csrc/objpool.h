// objpool.h -- per-thread recycling of the control plane's fixed-size heap
// objects (window subwindows, recovery-list nodes).  A bench step creates and
// frees thousands of codecs, each owning dozens of these; recycling them keeps
// the C heap (whose cross-thread frees contend on its arena locks) out of the
// hot path.  An object freed on one thread is reused by that thread.
#pragma once

#include <cstddef>
#include <mutex>
#include <new>
#include <vector>

namespace sgpu {

/// Objects taken on one thread are often put back on another (a decoder's
/// recovery packets are added on the thread that steps it and freed on the
/// one that finishes it), so each thread keeps at most kLocal and the rest
/// circulate through a shared depot in batches of kBatch (one lock per batch),
/// as RawPool below: a thread whose own stash ran dry refills from it instead
/// of calling the C heap (12 % of recovery packets did, before the depot).
template <class T>
class ObjPool
{
public:
    static T* get()
    {
        Stash& s = stash();
        if (s.items.empty())
            refill(s);
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
        if (s.items.size() >= kLocal)
            spill(s);
        s.items.push_back(p);
    }

private:
    static constexpr size_t kLocal = 2048;
    static constexpr size_t kBatch = kLocal / 2;
    static constexpr size_t kDepotMax = 1u << 16;
    struct Depot
    {
        std::mutex mu;
        std::vector<T*> items;
    };
    static Depot& depot()
    {
        static Depot* d = new Depot;   // (never destroyed: threads may exit after static teardown)
        return *d;
    }
    struct Stash
    {
        std::vector<T*> items;
        ~Stash()
        {
            Depot& d = depot();
            std::lock_guard<std::mutex> g(d.mu);
            for (T* p : items) {
                if (d.items.size() < kDepotMax)
                    d.items.push_back(p);
                else
                    delete p;
            }
        }
    };
    static void spill(Stash& s)
    {
        Depot& d = depot();
        std::lock_guard<std::mutex> g(d.mu);
        for (size_t k = 0; k < kBatch; ++k) {
            T* p = s.items.back();
            s.items.pop_back();
            if (d.items.size() < kDepotMax)
                d.items.push_back(p);
            else
                delete p;
        }
    }
    static void refill(Stash& s)
    {
        Depot& d = depot();
        std::lock_guard<std::mutex> g(d.mu);
        const size_t n = d.items.size() < kBatch ? d.items.size() : kBatch;
        s.items.insert(s.items.end(), d.items.end() - (long)n, d.items.end());
        d.items.resize(d.items.size() - n);
    }
    static Stash& stash()
    {
        thread_local Stash s;
        return s;
    }
};

/// Per-thread recycling of raw storage for objects of type T (the codec
/// instances themselves: 1.5-2.5 KB each, past the C heap's per-thread
/// caches, so every create and free would take an arena lock -- contended,
/// since instances are created and freed on different threads).  get()
/// returns uninitialised storage (construct with placement new); put() takes
/// storage whose object was destroyed.  A thread keeps at most kLocal blocks;
/// past that, half of them move to a shared depot (one lock per kBatch
/// blocks), which a thread whose own stash is empty drains first.  Instances
/// created on one thread and freed on another therefore circulate instead of
/// piling up in the freeing thread's stash.
template <class T>
class RawPool
{
public:
    static void* get()
    {
        Stash& s = stash();
        if (s.items.empty())
            refill(s);
        if (!s.items.empty()) {
            void* p = s.items.back();
            s.items.pop_back();
            return p;
        }
        return ::operator new(sizeof(T), std::align_val_t(alignof(T) > 64 ? alignof(T) : 64), std::nothrow);
    }
    static void put(void* p)
    {
        Stash& s = stash();
        if (s.items.size() >= kLocal)
            spill(s);
        s.items.push_back(p);
    }

private:
    static constexpr size_t kLocal = 256;
    static constexpr size_t kBatch = kLocal / 2;
    static constexpr size_t kDepotMax = 1u << 14;   // blocks the depot keeps at most
    static void release(void* p)
    {
        ::operator delete(p, std::align_val_t(alignof(T) > 64 ? alignof(T) : 64));
    }
    struct Depot
    {
        std::mutex mu;
        std::vector<void*> items;
    };
    static Depot& depot()
    {
        static Depot* d = new Depot;   // (never destroyed: threads may exit after static teardown)
        return *d;
    }
    struct Stash
    {
        std::vector<void*> items;
        ~Stash()
        {
            // back to the depot for the threads still running
            Depot& d = depot();
            std::lock_guard<std::mutex> g(d.mu);
            for (void* p : items) {
                if (d.items.size() < kDepotMax)
                    d.items.push_back(p);
                else
                    release(p);
            }
        }
    };
    static void spill(Stash& s)
    {
        Depot& d = depot();
        std::lock_guard<std::mutex> g(d.mu);
        for (size_t k = 0; k < kBatch; ++k) {
            void* p = s.items.back();
            s.items.pop_back();
            if (d.items.size() < kDepotMax)
                d.items.push_back(p);
            else
                release(p);
        }
    }
    static void refill(Stash& s)
    {
        Depot& d = depot();
        std::lock_guard<std::mutex> g(d.mu);
        const size_t n = d.items.size() < kBatch ? d.items.size() : kBatch;
        s.items.insert(s.items.end(), d.items.end() - (long)n, d.items.end());
        d.items.resize(d.items.size() - n);
    }
    static Stash& stash()
    {
        thread_local Stash s;
        return s;
    }
};

/// Per-thread stash of objects that hold reusable heap capacity (cleared
/// vectors) for the next instance of a codec created on the same thread, and
/// of the empty shells such an object leaves once its capacity is taken.
template <class T>
class CapStash
{
public:
    /// An object holding capacity, or null.
    static T* take()
    {
        Lists& l = lists();
        if (l.full.empty())
            return nullptr;
        T* p = l.full.back();
        l.full.pop_back();
        return p;
    }
    static void give(T* p)
    {
        Lists& l = lists();
        if (l.full.size() < kMax)
            l.full.push_back(p);
        else
            delete p;
    }
    /// An object whose members are all empty (to fill and give back).
    static T* shell()
    {
        Lists& l = lists();
        if (l.shells.empty())
            return new T;
        T* p = l.shells.back();
        l.shells.pop_back();
        return p;
    }
    static void put_shell(T* p)
    {
        Lists& l = lists();
        if (l.shells.size() < kMax)
            l.shells.push_back(p);
        else
            delete p;
    }

private:
    static constexpr size_t kMax = 1u << 12;
    struct Lists
    {
        std::vector<T*> full, shells;
        ~Lists()
        {
            for (T* p : full)
                delete p;
            for (T* p : shells)
                delete p;
        }
    };
    static Lists& lists()
    {
        thread_local Lists l;
        return l;
    }
};

} // namespace sgpu
