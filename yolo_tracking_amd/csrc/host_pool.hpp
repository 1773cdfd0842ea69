// Persistent host worker threads for the host-buffer ABI's staging copies (pageable caller
// buffers <-> pinned staging buffers).  One pool per engine, created on the first large copy and
// joined when the engine is destroyed; a copy is split into one piece per thread, the calling
// thread copying piece 0.  Replaces spawning and joining threads for every staging chunk.
#pragma once

#include <algorithm>
#include <condition_variable>
#include <cstddef>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

class CopyPool {
public:
    explicit CopyPool(int workers) {
        th_.reserve(workers);
        for (int k = 0; k < workers; ++k) th_.emplace_back([this, k] { run(k); });
    }
    ~CopyPool() {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_work_.notify_all();
        for (auto &t : th_) t.join();
    }
    CopyPool(const CopyPool &) = delete;
    CopyPool &operator=(const CopyPool &) = delete;

    int threads() const { return (int)th_.size() + 1; }

    // memcpy(dst, src, bytes) split into `parts` pieces (1 <= parts <= threads()).
    void copy(void *dst, const void *src, size_t bytes, int parts) {
        parts = std::max(1, std::min(parts, threads()));
        if (parts == 1) {
            memcpy(dst, src, bytes);
            return;
        }
        const size_t piece = (bytes + parts - 1) / parts;
        {
            std::lock_guard<std::mutex> lk(m_);
            dst_ = (char *)dst;
            src_ = (const char *)src;
            bytes_ = bytes;
            piece_ = piece;
            parts_ = parts;
            pending_ = (int)th_.size();
            ++gen_;
        }
        cv_work_.notify_all();
        memcpy(dst, src, std::min(piece, bytes));
        std::unique_lock<std::mutex> lk(m_);
        cv_done_.wait(lk, [this] { return pending_ == 0; });
    }

private:
    void run(int k) {
        unsigned long long seen = 0;
        for (;;) {
            std::unique_lock<std::mutex> lk(m_);
            cv_work_.wait(lk, [&] { return stop_ || gen_ != seen; });
            if (stop_) return;
            seen = gen_;
            const int part = k + 1;
            char *d = dst_;
            const char *s = src_;
            const size_t bytes = bytes_, piece = piece_;
            const bool mine = part < parts_;
            lk.unlock();
            if (mine) {
                const size_t o = (size_t)part * piece;
                if (o < bytes) memcpy(d + o, s + o, std::min(piece, bytes - o));
            }
            lk.lock();
            if (--pending_ == 0) cv_done_.notify_one();
        }
    }

    std::vector<std::thread> th_;
    std::mutex m_;
    std::condition_variable cv_work_, cv_done_;
    char *dst_ = nullptr;
    const char *src_ = nullptr;
    size_t bytes_ = 0, piece_ = 0;
    int parts_ = 0, pending_ = 0;
    unsigned long long gen_ = 0;
    bool stop_ = false;
};
